"""GPU tests of the rest of the routing_filter.h boundary:
routing_filter_estimate_unique_fp (host images and device-resident batches),
routing_filter_lookup_async, routing_filter_verify, estimate_unique_keys -- each against the
oracle or the committed golden fixtures, through the C ABI."""
import threading

import numpy as np
import pytest

from splinterdb_amd import engine as E
from splinterdb_amd import keys as K

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def test_estimate_unique_fp_chain_golden(golden_filters, oracle):
    """The filter_test-style incremental chain (4 values): the GPU estimate over the four
    GPU-built images equals the golden value recorded from the oracle."""
    z = golden_filters
    cfg = E.routing_config_init()
    filt, chain = None, []
    for i in range(4):
        filt = E.routing_filter_add(cfg, filt, z[f"chain_v{i}/hashes"], value=i)
        chain.append(filt)
    assert E.routing_filter_estimate_unique_fp(cfg, chain) == int(z["chain/estimate_unique_fp"][0])


def _mixed_set(oracle, lis=8):
    """Filters of several sizes/values, one with < 16 indices (skipped by the reference), and
    a NULL filter; returns (engine images, oracle filters, hashes per filter)."""
    cfg = E.routing_config_init(log_index_size=lis)
    ocfg = oracle.make_config(log_index_size=lis)
    sizes = [1 << 20, 100_000, 3000, 700_000, 0, 2_000_000]
    vals = [0, 3, 1, 17, 0, 5]
    imgs, ofs, hs = [], [], []
    for j, (n, v) in enumerate(zip(sizes, vals)):
        if n == 0:
            imgs.append(None)
            ofs.append(None)
            hs.append(None)
            continue
        # overlapping key ranges, so the union has shared fingerprints
        h = oracle.hash_fixed(K.seq_keys(j * 50_000, n).reshape(-1), 24)
        imgs.append(E.routing_filter_add(cfg, None, h, value=v))
        ofs.append(oracle.filter_add(ocfg, h, value=v))
        hs.append(h)
    return cfg, ocfg, imgs, ofs, hs


def test_estimate_unique_fp_matches_oracle(oracle):
    cfg, ocfg, imgs, ofs, _ = _mixed_set(oracle)
    want = oracle.estimate_unique_fp(ocfg, ofs)
    assert want > 0
    assert E.routing_filter_estimate_unique_fp(cfg, imgs) == want
    # subsets, including a single filter and an all-NULL list
    for sub in ([0], [1, 2], [2], [4], [0, 3, 5], []):
        assert E.routing_filter_estimate_unique_fp(cfg, [imgs[i] for i in sub]) == \
            oracle.estimate_unique_fp(ocfg, [ofs[i] for i in sub]), sub


def test_batch_estimate_unique_fp_matches_oracle(oracle):
    """Device-resident images (no host round trip), two batches mixed."""
    cfg = E.routing_config_init()
    ocfg = oracle.make_config()
    sizes_a, vals_a = [1 << 20, 300_000, 5000], [0, 2, 9]
    sizes_b, vals_b = [800_000], [4]
    ka = K.random_keys(sum(sizes_a), seed=11)
    kb = K.random_keys(sum(sizes_b), seed=11)  # same first keys: shared fingerprints
    ba, bb = E.FilterBatch(cfg, sizes_a, vals_a), E.FilterBatch(cfg, sizes_b, vals_b)
    ba.build_keys(dev(ka), 24)
    bb.build_keys(dev(kb), 24)
    ofs, s = [], 0
    ha = oracle.hash_fixed(ka.reshape(-1), 24)
    for n, v in zip(sizes_a, vals_a):
        ofs.append(oracle.filter_add(ocfg, ha[s:s + n], value=v))
        s += n
    ofs.append(oracle.filter_add(ocfg, oracle.hash_fixed(kb.reshape(-1), 24), value=vals_b[0]))
    members = [(ba, 0), (ba, 1), (ba, 2), (bb, 0), None]
    want = oracle.estimate_unique_fp(ocfg, ofs + [None])
    assert E.batch_estimate_unique_fp(members) == want
    assert E.batch_estimate_unique_fp([(ba, 0), (bb, 0)]) == oracle.estimate_unique_fp(ocfg, [ofs[0], ofs[3]])


def test_estimate_unique_fp_error_contract(oracle):
    cfg = E.routing_config_init()
    f = E.routing_filter_add(cfg, None, oracle.hash_fixed(K.seq_keys(0, 70_000).reshape(-1), 24))
    with pytest.raises(E.PlatformStatusError) as ei:  # > MAX_FILTERS (:717)
        E.routing_filter_estimate_unique_fp(cfg, [f] * 33)
    assert ei.value.code == E.STATUS_BAD_PARAM
    # every fingerprint in the first 1/16 of the indices: the reference's num_fp/12 buffer
    # overflows and it asserts (:776); lis 6 keeps each index under 4096 entries
    cfg6 = E.routing_config_init(log_index_size=6)
    ocfg6 = oracle.make_config(log_index_size=6)
    h = (K.splitmix64(7, 50_000) & np.uint64(0x0FFFFFFF)).astype(np.uint32)
    g = E.routing_filter_add(cfg6, None, h)
    with pytest.raises(ValueError):
        oracle.estimate_unique_fp(ocfg6, [oracle.filter_add(ocfg6, h)])
    with pytest.raises(E.PlatformStatusError) as ei:
        E.routing_filter_estimate_unique_fp(cfg6, [g])
    assert ei.value.code == E.STATUS_BAD_PARAM


def test_estimate_unique_keys(oracle):
    cfg = E.routing_config_init()
    f = E.routing_filter_add(cfg, None, oracle.hash_fixed(K.seq_keys(0, 1_000_000).reshape(-1), 24))
    assert f.num_unique == 992_680  # SURVEY.md §8(c) known answer
    assert E.routing_filter_estimate_unique_keys(f, cfg) == \
        oracle.estimate_unique_keys_from_count(oracle.make_config(), f.num_unique)


def test_lookup_async_matches_sync_probe(oracle):
    """rf_amd_lookup_async (routing_filter_lookup_async, routing_filter.h:130-155) returns the
    oracle's routing_filter_lookup of every probe in its filter, and fires its callback."""
    cfg = E.routing_config_init()
    sizes, vals = [200_000, 50_000, 123_457], [0, 7, 63 - 32]
    keys = K.random_keys(sum(sizes), seed=5)
    b = E.FilterBatch(cfg, sizes, vals)
    b.build_keys(dev(keys), 24)
    # probes: the inserted keys (routed to their filter) plus negatives routed anywhere
    neg = K.random_keys(100_000, seed=6)
    pk = np.concatenate([keys, neg])
    fid = np.concatenate([np.repeat(np.arange(3, dtype=np.uint32), sizes),
                          (np.arange(100_000) % 3).astype(np.uint32)])
    found = torch.zeros(pk.shape[0], dtype=torch.int64, device="cuda:0")
    b.probe_keys(dev(pk), 24, dev(fid), pk.shape[0], found)
    torch.cuda.synchronize()
    want = found.cpu().numpy().view(np.uint64)
    ocfg = oracle.make_config()
    starts = np.cumsum([0] + sizes)
    ph = oracle.hash_fixed(pk.reshape(-1), 24)
    for i in range(3):
        of = oracle.filter_add(ocfg, oracle.hash_fixed(keys[starts[i]:starts[i + 1]].reshape(-1), 24),
                               value=vals[i])
        sel = fid == i
        assert (of.lookup_hashes(ph[sel]) == want[sel]).all()
    fired = threading.Event()
    la = E.LookupAsync(b, pk, fid, callback=fired.set)
    got = la.wait()
    assert fired.wait(10)
    assert la.poll() == E.ASYNC_STATUS_DONE
    assert (got == want).all()
    la.close()
    # filter_id omitted: every probe goes to filter 0
    la0 = E.LookupAsync(b, keys[: sizes[0]])
    assert ((la0.wait() & np.uint64(1)) == 1).all()
    la0.close()


def test_verify(oracle):
    cfg = E.routing_config_init()
    keys = K.random_keys(300_000, seed=9)
    f = E.routing_filter_add(cfg, None, oracle.hash_fixed(keys.reshape(-1), 24), value=3)
    assert E.routing_filter_verify(cfg, f, keys, 3) == 0
    with pytest.raises(E.PlatformStatusError) as ei:
        E.routing_filter_verify(cfg, f, keys, 4)
    assert ei.value.code == E.STATUS_BAD_PARAM and ei.value.num_missing == 300_000


def test_hash_keys_match_oracle(oracle):
    """rf_amd_hash_keys / _var_keys: XXH32 (seed from the config) of device-resident keys."""
    for key_len in (24, 16, 7, 100):
        keys = K.random_keys(50_000, key_len=key_len, seed=key_len)
        out = torch.zeros(50_000, dtype=torch.int32, device="cuda:0")
        E.hash_keys(E.routing_config_init(seed=7), dev(keys), key_len, 50_000, out)
        torch.cuda.synchronize()
        assert (out.cpu().numpy().view(np.uint32) == oracle.hash_fixed(keys.reshape(-1), key_len, seed=7)).all()
    d, o = K.var_keys(30_000)
    out = torch.zeros(30_000, dtype=torch.int32, device="cuda:0")
    E.hash_var_keys(E.routing_config_init(), dev(d), dev(o), 30_000, out)
    torch.cuda.synchronize()
    assert (out.cpu().numpy().view(np.uint32) == oracle.hash_var(d, o)).all()


@pytest.mark.gpu
def test_probe_runs_equal_per_probe_filter_ids(oracle):
    """rf_amd_batch_probe_{keys,hashes}_runs (filter from the probe's position) must equal the
    per-probe filter-id probe, including empty runs and runs longer than the filter."""
    from splinterdb_amd import keys as K
    cfg = E.routing_config_init()
    sizes, vals = [20000, 1, 70000, 3000, 9], [1, 0, 4, 2, 7]
    b = E.FilterBatch(cfg, sizes, vals)
    b.build_keys(torch.from_numpy(K.seq_keys(0, sum(sizes)).reshape(-1)).to("cuda:0"), 24)
    rng = np.random.default_rng(3)
    counts = [5000, 0, 100000, 17, 4099]
    ids = rng.integers(0, 2 * sum(sizes), size=sum(counts)).astype(np.uint64)
    fid = np.repeat(np.arange(len(counts), dtype=np.uint32), counts)
    keys = torch.from_numpy(K.ids_keys(ids).reshape(-1)).to("cuda:0")
    P = len(ids)
    f_ids = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    f_runs = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b.probe_keys(keys, 24, torch.from_numpy(fid.view(np.int32)).to("cuda:0"), P, f_ids)
    b.probe_keys_runs(keys, 24, counts, f_runs)
    torch.cuda.synchronize()
    assert torch.equal(f_ids, f_runs)
    h = oracle.hash_fixed(K.ids_keys(ids).reshape(-1), 24)
    f_h = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b.probe_hashes_runs(torch.from_numpy(h.view(np.int32)).to("cuda:0"), counts, f_h)
    counts2 = [1, 1, 1, 1, P - 4]  # a second shape: the bounds are re-uploaded
    f_r2 = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b.probe_keys_runs(keys, 24, counts2, f_r2)
    fid2 = np.repeat(np.arange(5, dtype=np.uint32), counts2)
    f_i2 = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b.probe_keys(keys, 24, torch.from_numpy(fid2.view(np.int32)).to("cuda:0"), P, f_i2)
    torch.cuda.synchronize()
    assert torch.equal(f_ids, f_h)
    assert torch.equal(f_r2, f_i2)
    # and both shapes equal the oracle's routing_filter_lookup of each probe in its filter
    # (runs crossing waves, empty runs, and waves spanning five filters: the wave table path)
    ocfg = oracle.make_config()
    starts = np.cumsum([0] + sizes)
    ofs = [oracle.filter_add(ocfg, oracle.hash_fixed(K.seq_keys(int(starts[i]), sizes[i]).reshape(-1), 24),
                             value=vals[i]) for i in range(len(sizes))]
    for cs, got in ((counts, f_runs), (counts2, f_r2)):
        want = np.zeros(P, dtype=np.uint64)
        at = 0
        for i, c in enumerate(cs):
            if c:
                want[at:at + c] = ofs[i].lookup_hashes(h[at:at + c])
            at += c
        assert (got.cpu().numpy().view(np.uint64) == want).all()
