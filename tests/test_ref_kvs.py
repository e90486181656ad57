"""The reference's whole key-value store (splinterdb.c / core.c / trunk.c / btree.c / ...,
compiled unmodified, oracle/ref_kvs.c) as the routing filter's caller, on the CPU with the
reference's own routing_filter.c: the harness itself is checked here (a shadow of every
insert, sync and async lookups, the filter adds the trunk makes), so the GPU test that runs
the same workload on the drop-in (tests/test_gpu_trunk.py) compares two working stacks."""
import numpy as np
import pytest

from oracle import refkvs as RK
from splinterdb_amd import keys as K

pytestmark = pytest.mark.skipif(not RK.available(RK.KVS_REF), reason="oracle/_ref/libkvs_ref.so not built")


def workload(n, seed=7):
    """n distinct 24-byte keys in a scattered order (filter_test's id format), 8-byte values;
    absent keys of the same form"""
    rng = np.random.default_rng(seed)
    ids = rng.permutation(np.arange(n, dtype=np.uint64)) * np.uint64(7919) + np.uint64(13)
    keys = K.ids_keys(ids)
    vals = (ids * np.uint64(0x9E3779B97F4A7C15)).view(np.uint8).reshape(n, 8)
    absent = K.ids_keys(np.arange(n, dtype=np.uint64) * np.uint64(7919) + np.uint64(14))
    return keys, vals, absent


def test_reference_kvstore_shadow_and_filter_calls():
    """300,000 inserts through splinterdb_insert (2 MiB memtables: flushes and trunk
    compactions), then every key found with its value and 30,000 absent keys not found,
    synchronously (splinterdb_lookup) and through core_lookup_async with 64 in flight; the
    trunk built its maplets with routing_filter_add, some incrementally (old filter), and
    looked them up with routing_filter_lookup / _lookup_async"""
    n = 300_000
    keys, vals, absent = workload(n)
    with RK.Kvs(RK.KVS_REF, memtable_mib=2) as db:
        db.insert(keys, vals)
        recs, _, _ = db.adds()
        assert len(recs) >= 5
        assert (recs["rc"] == 0).all()
        assert (recs["old_addr"] != 0).any()  # incremental adds (maplet compaction onto the old maplet)
        assert (recs["num_fingerprints"] > 0).all() and (recs["digest"] != 0).all()
        sample = np.random.default_rng(1).choice(n, 30_000, replace=False)
        f, v, _ = db.lookup(keys[sample])
        assert f.all()
        assert (v == vals[sample].view(np.uint64).ravel()).all()
        fa, va, _ = db.lookup(absent[:30_000])
        assert not fa.any()
        f2, v2, _ = db.lookup_async(np.concatenate([keys[sample], absent[:30_000]]), 64)
        assert (f2[:30_000]).all() and not f2[30_000:].any()
        assert (v2[:30_000] == v).all()
        _, nl, na = db.adds()
        assert nl > 0 and na > 0
