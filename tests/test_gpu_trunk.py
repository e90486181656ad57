"""The reference's own trunk as the drop-in's caller, on the GPU.

The reference's whole key-value store (splinterdb.c, core.c, trunk.c, btree.c, memtable.c, ...,
compiled unmodified; oracle/ref_kvs.c) runs the same workload twice: linked with the
reference's routing_filter.c (oracle/_ref/libkvs_ref.so) and with shim/routing_filter_amd.c
(oracle/_ref/libkvs_shim.so, building and probing on the MI355X). Every routing_filter_add the
trunk's compactions make (maplet_compaction_task, src/trunk.c:3780-3927) must return the same
descriptor and the same bytes (index slots and data pages, read back through the cache), and
every lookup -- splinterdb_lookup, which reaches routing_filter_lookup through
trunk_ondisk_bundle_merge_lookup (:6008-6110), and core_lookup_async, which reaches
routing_filter_lookup_async (:6136) -- must return the same result, equal to a shadow of the
inserts (tests/functional/test_functionality.c's check)."""
import numpy as np
import pytest

from oracle import refkvs as RK
from test_ref_kvs import workload

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (RK.available(RK.KVS_REF) and RK.available(RK.KVS_SHIM)),
                                 reason="oracle/_ref/libkvs_{ref,shim}.so not built")]


def run(path, keys, vals, probe, memtable_mib, attach=True, stats=None):
    with RK.Kvs(path, memtable_mib=memtable_mib, attach=attach) as db:
        if stats is not None:
            stats.append(db.direct_stats())
        db.insert(keys, vals)
        recs, nl0, na0 = db.adds()
        f, v, _ = db.lookup(probe)
        fa, va, _ = db.lookup_async(probe, 64)
        _, nl, na = db.adds()
    return recs, (f, v), (fa, va), nl - nl0, na - na0


@pytest.mark.parametrize("n,memtable_mib", [(400_000, 2), (1_200_000, 4)])
def test_trunk_filters_and_lookups_identical_to_reference(n, memtable_mib):
    keys, vals, absent = workload(n, seed=n)
    rng = np.random.default_rng(3)
    sample = rng.choice(n, 40_000, replace=False)
    probe = np.concatenate([keys[sample], absent[:40_000]])
    ref = run(RK.KVS_REF, keys, vals, probe, memtable_mib)
    shim = run(RK.KVS_SHIM, keys, vals, probe, memtable_mib)
    # the same routing_filter_add calls with the same results, byte for byte
    assert len(ref[0]) == len(shim[0]) and len(ref[0]) > 5
    for i, (a, b) in enumerate(zip(ref[0], shim[0])):
        assert a.tolist() == b.tolist(), (i, dict(zip(RK.ADD_FIELDS, a.tolist())), dict(zip(RK.ADD_FIELDS, b.tolist())))
    want_v = vals[sample].view(np.uint64).ravel()
    for (f, v) in (ref[1], ref[2], shim[1], shim[2]):
        assert f[:40_000].all() and not f[40_000:].any()  # the shadow
        assert (v[:40_000] == want_v).all()
    # the same filter calls reached the filter (the trunk prunes by the filter's answers)
    assert ref[3] == shim[3] and ref[4] == shim[4]


@pytest.mark.parametrize("attach", [False, True])
def test_reopened_stores_filters_identical(attach):
    """Three stores opened and closed one after another in one process (their cache buffers
    may be mapped again at the same address with the same size). attach=False drives them as
    the unmodified reference does -- no shim extension called, so no cache is registered and
    every image takes the bounce-buffer path; attach=True attaches each store's cache after
    opening and releases it before closing (direct placement). Either way each store gets the
    reference's filters byte for byte and its lookups."""
    stats = []
    for i, seed in enumerate((21, 22, 23)):
        keys, vals, absent = workload(300_000, seed=seed)
        probe = np.concatenate([keys[:20_000], absent[:20_000]])
        ref = run(RK.KVS_REF, keys, vals, probe, 2, attach=False)
        shim = run(RK.KVS_SHIM, keys, vals, probe, 2, attach=attach, stats=stats)
        assert len(ref[0]) == len(shim[0]) and len(ref[0]) > 3
        for j, (a, b) in enumerate(zip(ref[0], shim[0])):
            assert a.tolist() == b.tolist(), (i, j)
        for (f, v), (g, w) in ((ref[1], shim[1]), (ref[2], shim[2])):
            assert (f == g).all() and (v == w).all(), i
    # (caches registered, stale placements, adds placing) while each store was open
    assert all(s[0] == (1 if attach else 0) and s[1] == 0 for s in stats), stats
