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
    then polled: the shim submits them to the engine's lookup server (every first call returns
    ASYNC_STATUS_RUNNING; 20,000 states wrap its 4,096-slot ring several times) and its
    completion thread reaps the answers; every found_values equals the reference coroutine's,
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
    # every state was queued (its first call returned RUNNING, never DONE) and completed by
    # a flush with its callback fired exactly once
    assert cb_s == P and run_s == P
    assert p1 - p0 == P and 0 < b1 - b0 <= P  # reaped in batches
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


@pytest.mark.parametrize("inflight", [1, 64, 4096])
def test_lookup_async_callback_driven(pair, inflight):
    """routing_filter_lookup_async driven as tests/functional/test_async.c drives it: a state
    is called again only after its callback fired (async_ctxt_process_ready, :168-196). Every
    queued state must complete without being called again (the shim's completion thread), a
    call never both fires its state's callback and returns DONE, each waiting state gets
    exactly one callback, and every result equals the reference coroutine's"""
    ref, shim = pair
    descs_r, descs_s, allkeys = [], [], []
    for f, n in enumerate((30_000, 5_000)):
        keys = K.random_keys(n, seed=300 + f)
        h = ref.hash_keys(keys)
        descs_r.append(ref.add(h, value=f + 2))
        descs_s.append(shim.add(h, value=f + 2))
        allkeys.append(keys)
    rng = np.random.default_rng(9)
    P = 6000 if inflight == 1 else 20_000
    fid = rng.integers(0, 2, size=P).astype(np.uint32)
    probe = K.random_keys(P, seed=0xCB)
    for i in np.nonzero(rng.random(P) < 0.6)[0]:
        src = allkeys[fid[i]]
        probe[i] = src[rng.integers(0, src.shape[0])]
    want, st_r = ref.lookup_keys_async_driven(descs_r, probe, fid, max_inflight=inflight)
    got, st_s = shim.lookup_keys_async_driven(descs_s, probe, fid, max_inflight=inflight)
    assert (got == want).all()
    assert st_r == {"running": 0, "callbacks": 0, "done": P, "violations": 0}  # all cached
    assert st_s == {"running": P, "callbacks": P, "done": P, "violations": 0}, st_s


def test_async_states_over_512_filters_then_flush(pair):
    """8,192 async states over 512 distinct filters, all submitted to the engine's lookup
    server, then routing_filter_amd_flush(): every state is done once the flush returns, each
    callback fired once, and every result equals the reference's lookups"""
    ref, shim = pair
    descs_r, descs_s, allkeys = [], [], []
    for f in range(512):
        keys = K.ids_keys((np.uint64(f) << np.uint64(32)) + np.arange(500 + f, dtype=np.uint64))
        h = ref.hash_keys(keys)
        descs_r.append(ref.add(h, value=f % 40))
        descs_s.append(shim.add(h, value=f % 40))
        allkeys.append(keys)
    rng = np.random.default_rng(11)
    P = 8192
    fid = rng.integers(0, 512, size=P).astype(np.uint32)
    probe = K.random_keys(P, seed=0x512)
    for i in np.nonzero(rng.random(P) < 0.5)[0]:
        src = allkeys[fid[i]]
        probe[i] = src[rng.integers(0, src.shape[0])]
    want, _ = ref.lookup_batch(descs_r, probe, fid)
    b0, p0 = shim.async_stats()
    got, cb = shim.lookup_keys_async_flush(descs_s, probe, fid)
    b1, p1 = shim.async_stats()
    assert cb == P
    assert p1 - p0 == P and 0 < b1 - b0 <= P
    assert (got == want).all()


def test_async_states_of_two_routing_configs_in_one_flush():
    """Two kvstores with different filter_hash_size / filter_log_index_size
    (splinterdb.c:147-152) share the drop-in: async states of both go to the engine's lookup
    server together (each filter probed with its own routing config) and one flush completes
    them; every result equals the reference's (a launch used to reject mixed
    configs)"""
    cfgs = ((26, 8), (20, 6))
    refs = [R.Stack(fingerprint_size=a, log_index_size=b, cache_mib=512, disk_mib=4096) for a, b in cfgs]
    shims = [R.Stack(fingerprint_size=a, log_index_size=b, cache_mib=512, disk_mib=4096, path=R.SHIM_PATH)
             for a, b in cfgs]
    try:
        descs_r, descs_s, owner, allkeys = [], [], [], []
        for f, n in enumerate((40_000, 9_000, 25_000, 3)):
            st = f % 2
            keys = K.random_keys(n, seed=700 + f)
            h = refs[st].hash_keys(keys)
            descs_r.append(refs[st].add(h, value=f + 1))
            descs_s.append(shims[st].add(h, value=f + 1))
            owner.append(st)
            allkeys.append(keys)
        rng = np.random.default_rng(21)
        P = 12_000
        fid = rng.integers(0, len(descs_s), size=P).astype(np.uint32)
        probe = K.random_keys(P, seed=0x2CF)
        for i in np.nonzero(rng.random(P) < 0.6)[0]:
            src = allkeys[fid[i]]
            probe[i] = src[rng.integers(0, src.shape[0])]
        want = np.zeros(P, dtype=np.uint64)
        for f, d in enumerate(descs_r):
            m = fid == f
            want[m] = refs[owner[f]].lookup_keys(d, probe[m])
        sh = shims[0]
        b0, p0 = sh.async_stats()
        got, cb = sh.lookup_keys_async_flush_multi(shims, descs_s, owner, probe, fid)
        b1, p1 = sh.async_stats()
        assert cb == P
        assert p1 - p0 == P and 0 < b1 - b0 <= P
        assert (got == want).all()
        for st in refs + shims:
            assert st.device_writes() == 0
    finally:
        for st in refs + shims:
            st.close()


def test_concurrent_adds_and_lookups_from_8_threads(pair):
    """8 registered threads at once, each growing its own filter by 3 incremental
    routing_filter_add calls (2^17 keys each) and then looking up 4,000 keys synchronously
    and through async states -- SplinterDB's TASK_TYPE_NORMAL workers compacting different
    branches (src/trunk.c:3932, :4168). Concurrent adds are coalesced into shared GPU batches;
    every filter's image equals the reference's single-threaded build of the same chain
    (addresses depend on the threads' interleaving in both libraries, bytes do not), and
    every lookup equals the reference's."""
    ref, shim = pair
    T, R, n, NP = 8, 3, 1 << 17, 4000
    ids = np.arange(T * R * n, dtype=np.uint64) * np.uint64(2654435761) % np.uint64(1 << 40)
    keys = K.ids_keys(ids)
    rng = np.random.default_rng(5)
    kt = keys.reshape(T, R * n, 24)
    probe = np.concatenate([np.concatenate([kt[t][rng.integers(0, R * n, NP // 2)],
                                            K.random_keys(NP // 2, seed=70 + t)]) for t in range(T)])
    s0 = shim.shim_stats()
    chains, fs, fa, add_s = shim.mt_chains(keys, T, R, n, probe, NP)
    s1 = shim.shim_stats()
    assert s1["add_filters"] - s0["add_filters"] == T * R
    assert s1["add_batches"] - s0["add_batches"] <= T * R
    kr = keys.reshape(T, R, n, 24)
    for t in range(T):
        old = None
        for r in range(R):
            old = ref.add(ref.hash_keys(kr[t, r]), value=r, old=old)
            ir, is_ = ref.image(old), shim.image(chains[t][r])
            assert (ir.num_unique, ir.num_pages) == (is_.num_unique, is_.num_pages), (t, r)
            assert (ir.pages == is_.pages).all() and (ir.slots == is_.slots).all(), (t, r)
        want = ref.lookup_keys(old, probe[t * NP:(t + 1) * NP])
        assert (fs[t * NP:(t + 1) * NP] == want).all(), t
        assert (fa[t * NP:(t + 1) * NP] == want).all(), t


def test_registry_bound_evicts_and_reimports(pair):
    """the shim keeps built filters on the device up to its bound (RF_AMD_REGISTRY_MIB):
    shrinking the bound trims and evicts least recently used filters; lookups on evicted
    filters re-import them from the cache and still equal the reference's"""
    ref, shim = pair
    descs_r, descs_s, allkeys = [], [], []
    for f in range(24):
        keys = K.random_keys(1 << 16, seed=900 + f)
        h = ref.hash_keys(keys)
        descs_r.append(ref.add(h, value=f % 7))
        descs_s.append(shim.add(h, value=f % 7))
        allkeys.append(keys)
    s0 = shim.shim_stats()
    assert shim.registry_set_limit(8)  # 8 MiB: a few probe-only filters
    try:
        s1 = shim.shim_stats()
        assert s1["trims"] > s0["trims"] and s1["evictions"] > s0["evictions"]
        assert s1["registry_bytes"] <= 8 << 20
        for f in range(24):
            probe = np.concatenate([allkeys[f][:500], K.random_keys(500, seed=f)])
            assert (shim.lookup_keys(descs_s[f], probe) == ref.lookup_keys(descs_r[f], probe)).all(), f
        # incremental adds onto evicted filters decode the re-imported image
        h = ref.hash_keys(K.random_keys(5000, seed=0xE))
        dr = ref.add(h, value=9, old=descs_r[0])
        ds = shim.add(h, value=9, old=descs_s[0])
        assert_same_pages(ref, shim, dr, ds, "onto evicted")
    finally:
        shim.registry_set_limit(32768)


_BOUNCE_CHECK = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from oracle import refimpl as R
from splinterdb_amd import keys as K
ref, shim = R.Stack(), R.Stack(path=R.SHIM_PATH)
rng = np.random.default_rng(5)
prev_r = prev_s = None
for n, value in ((1, 0), (20_000, 3), (700_000, 3), (300_000, 9)):
    h = ref.hash_keys(K.random_keys(n, seed=int(rng.integers(1 << 30))))
    dr = ref.add(h, value=value, old=prev_r)
    ds = shim.add(h, value=value, old=prev_s)
    assert (dr.addr, dr.meta_head, dr.num_fingerprints, dr.num_unique) == \
           (ds.addr, ds.meta_head, ds.num_fingerprints, ds.num_unique), n
    for p in range(32):
        a = dr.addr + 4096 * p
        assert (ref.read_page(a) == shim.read_page(a)).all(), (n, p)
    ir, is_ = ref.image(dr), shim.image(ds)
    assert (ir.slots == is_.slots).all() and (ir.pages == is_.pages).all(), n
    prev_r, prev_s = dr, ds
assert ref.device_writes() == 0 and shim.device_writes() == 0
print("OK")
"""


@pytest.mark.parametrize("env", [{"RF_SHIM_DIRECT": "0"}, {"RF_SHIM_DIRECT": "0", "RF_SHIM_PINNED": "0"},
                                 {"RF_SHIM_DIRECT_MAX_MIB": "0"}])
def test_add_bounce_paths_identical_to_reference(env):
    """routing_filter_add's fallbacks when images cannot go straight into the cache pages
    (RF_SHIM_DIRECT=0, or a cache buffer over RF_SHIM_DIRECT_MAX_MIB): read back into a
    recycled pinned buffer, or into malloc'd memory after an engine-wide sync
    (RF_SHIM_PINNED=0), then copied page by page -- fresh and incremental
    adds, pages and index extents identical to the reference's (in a subprocess: the
    switches are read once per process)"""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    r = subprocess.run([sys.executable, "-c", _BOUNCE_CHECK, ROOT], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
