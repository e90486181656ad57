"""The drop-in at the reference's own interface, on the GPU.

Two copies of the reference's page stack (its clockcache, mini_allocator, rc_allocator and
harness, oracle/ref_harness.c): one linked with the reference's src/routing_filter.c
(oracle/_ref/libref_rf.so), one with shim/routing_filter_amd.c in its place, which builds
and probes on the MI355X through librf_amd.so (oracle/_ref/libshim_rf.so). The same calls
go to both -- routing_filter_add (fresh and incremental), routing_filter_lookup, the
routing_filter_lookup_async coroutine, routing_filter_estimate_unique_fp,
routing_filter_print -- and the results must be identical: filter descriptors (index
extent address, meta head, counts), every byte of every cache page the filter occupies
(the 32-page index extent with its absolute slots, and the data pages), lookup bit-vectors,
estimates and printed text.
"""
import numpy as np
import pytest

from oracle import refimpl as R
from splinterdb_amd import keys as K

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (R.available() and R.available(R.SHIM_PATH)),
                                 reason="oracle/_ref libraries not built")]


def desc_tuple(d):
    return (d.addr, d.meta_head, d.num_fingerprints, d.num_unique, d.value_size)


def assert_same_pages(ref, shim, dr, ds, tag):
    """the index extent and every data page, raw, at the same disk addresses"""
    assert desc_tuple(dr) == desc_tuple(ds), (tag, desc_tuple(dr), desc_tuple(ds))
    for p in range(32):
        a = dr.addr + 4096 * p
        assert (ref.read_page(a) == shim.read_page(a)).all(), (tag, "index page", p)
    ir, is_ = ref.image(dr), shim.image(ds)
    assert (ir.slots == is_.slots).all() and ir.num_pages == is_.num_pages, tag
    assert (ir.pages == is_.pages).all(), tag


@pytest.fixture()
def pair():
    ref = R.Stack()
    shim = R.Stack(path=R.SHIM_PATH)
    yield ref, shim
    assert ref.device_writes() == 0 and shim.device_writes() == 0
    ref.close()
    shim.close()


def test_add_and_lookup_identical_to_reference(pair):
    """fresh filters of 1 .. 8,000,000 fingerprints with values 0 / 5 / 31, then lookups
    of inserted and never-inserted keys through routing_filter_lookup"""
    ref, shim = pair
    rng = np.random.default_rng(1)
    for n, value in ((1, 0), (100, 5), (10_000, 0), (1_000_000, 31), (8_000_000, 0), (300_000, 7)):
        keys = K.random_keys(n, seed=int(rng.integers(1 << 30)))
        h = ref.hash_keys(keys)
        dr = ref.add(h, value=value)
        ds = shim.add(h, value=value)
        assert_same_pages(ref, shim, dr, ds, (n, value))
        probe = np.concatenate([keys[: min(n, 3000)], K.random_keys(3000, seed=0xBAD)])
        fr = ref.lookup_keys(dr, probe)
        fs = shim.lookup_keys(ds, probe)
        assert (fr == fs).all(), (n, value)
        assert ((fr[: min(n, 3000)] >> np.uint64(value)) & np.uint64(1)).all()


def test_incremental_chain_identical_to_reference(pair):
    """tests/functional/filter_test.c's basic pattern through both: 8 values x 1,048,575
    fingerprints, each routing_filter_add merging into the previous filter (old_filter,
    src/routing_filter.c:496-597), then estimate_unique_fp over the chain"""
    ref, shim = pair
    nf = 1_048_575
    oldr = olds = None
    chain_r, chain_s = [], []
    for i in range(8):
        keys = K.ids_keys((i + 1) * np.arange(nf, dtype=np.uint64))
        h = ref.hash_keys(keys)
        oldr = ref.add(h, value=i, old=oldr)
        olds = shim.add(h, value=i, old=olds)
        assert_same_pages(ref, shim, oldr, olds, ("chain", i))
        chain_r.append(oldr)
        chain_s.append(olds)
    assert oldr.num_unique == 4254486
    assert ref.estimate_unique_fp(chain_r) == shim.estimate_unique_fp(chain_s)
    unused = 9 * nf
    neg = K.ids_keys(np.arange(unused, unused + 200_000, dtype=np.uint64))
    assert (ref.lookup_keys(oldr, neg) == shim.lookup_keys(olds, neg)).all()


def test_lookup_async_coalesced_equals_reference(pair):
    """20,000 routing_filter_lookup_async states over three filters, each started once and
    then polled: the shim queues them (every first call returns ASYNC_STATUS_RUNNING) and
    answers them in a few GPU probes; every found_values equals the reference coroutine's,
    every callback fires once"""
    ref, shim = pair
    descs_r, descs_s, allkeys = [], [], []
    for f, n in enumerate((50_000, 200_000, 7)):
        keys = K.random_keys(n, seed=100 + f)
        h = ref.hash_keys(keys)
        descs_r.append(ref.add(h, value=f))
        descs_s.append(shim.add(h, value=f))
        allkeys.append(keys)
    rng = np.random.default_rng(3)
    P = 20_000
    fid = rng.integers(0, 3, size=P).astype(np.uint32)
    probe = K.random_keys(P, seed=0xABC)
    pos = rng.random(P) < 0.7
    for i in np.nonzero(pos)[0]:
        src = allkeys[fid[i]]
        probe[i] = src[rng.integers(0, src.shape[0])]
    want, cb_r, run_r = ref.lookup_keys_async_many(descs_r, probe, fid)
    b0, p0 = shim.async_stats()
    got, cb_s, run_s = shim.lookup_keys_async_many(descs_s, probe, fid)
    b1, p1 = shim.async_stats()
    assert (got == want).all()
    # every state was queued and completed by a flush with its callback fired; the states
    # whose arrival filled the queue (every 1024th) were flushed inside their own first call
    assert cb_s == P and run_s == P - P // 1024
    assert p1 - p0 == P and 0 < b1 - b0 <= P // 1024 + 1  # one GPU round trip per flush
    assert run_r == 0  # the reference's coroutine finds every page in the cache
    # and the synchronous form agrees with both
    for f in range(3):
        m = fid == f
        assert (shim.lookup_keys(descs_s[f], probe[m]) == want[m]).all()


def test_lookup_batch_equals_reference_lookups(pair):
    """routing_filter_amd_lookup_batch (the trunk_merge_lookup batch form): 30,000 lookups
    spread over five filters and a NULL filter, in one GPU round trip, equal the reference's
    routing_filter_lookup of each (filter, key)"""
    ref, shim = pair
    descs_r, descs_s, allkeys = [], [], []
    for f, n in enumerate((1000, 80_000, 300_000, 5, 40_000)):
        keys = K.random_keys(n, seed=200 + f)
        h = ref.hash_keys(keys)
        descs_r.append(ref.add(h, value=f))
        descs_s.append(shim.add(h, value=f))
        allkeys.append(keys)
    descs_r.append(R.RoutingFilter())  # NULL filter: finds nothing
    descs_s.append(R.RoutingFilter())
    rng = np.random.default_rng(5)
    P = 30_000
    fid = rng.integers(0, 6, size=P).astype(np.uint32)
    probe = K.random_keys(P, seed=0xBEE)
    for i in np.nonzero(rng.random(P) < 0.6)[0]:
        if fid[i] < 5:
            src = allkeys[fid[i]]
            probe[i] = src[rng.integers(0, src.shape[0])]
    want, batched_r = ref.lookup_batch(descs_r, probe, fid)
    got, batched_s = shim.lookup_batch(descs_s, probe, fid)
    assert batched_s and not batched_r
    assert (got == want).all()
    assert (got[fid == 5] == 0).all() and (got[fid < 5] != 0).sum() > 0.4 * P


def test_print_identical_to_reference(pair, capfd):
    """routing_filter_print (src/routing_filter.c:1259-1285): the same text, absolute
    addresses included"""
    ref, shim = pair
    for n, value in ((3000, 0), (40_000, 3)):
        h = ref.hash_keys(K.random_keys(n, seed=n))
        dr, ds = ref.add(h, value=value), shim.add(h, value=value)
        tr, ts = ref.print_text(dr), shim.print_text(ds)
        assert tr.count("--- Index") == len(ref.image(dr).slots)
        assert tr == ts


def test_dec_ref_releases_and_other_filters_stay(pair):
    """dec_ref to zero frees the reference's extents (and the shim's device copy); a later
    filter reuses the freed pages, and lookups of a surviving filter are unaffected"""
    ref, shim = pair
    ha = ref.hash_keys(K.random_keys(100_000, seed=1))
    hb = ref.hash_keys(K.random_keys(100_000, seed=2))
    a_r, a_s = ref.add(ha), shim.add(ha)
    b_r, b_s = ref.add(hb), shim.add(hb)
    ref.dec_ref(a_r)
    shim.dec_ref(a_s)
    hc = ref.hash_keys(K.random_keys(50_000, seed=3))
    c_r, c_s = ref.add(hc), shim.add(hc)
    assert desc_tuple(c_r) == desc_tuple(c_s)
    probe = K.random_keys(5000, seed=2)
    assert (ref.lookup_keys(b_r, probe) == shim.lookup_keys(b_s, probe)).all()
    assert (ref.lookup_keys(c_r, probe) == shim.lookup_keys(c_s, probe)).all()
