"""Randomised GPU parity sweep: seeded random geometries (fingerprint_size, log_index_size),
sizes, values, incremental adds over an old filter, duplicate-heavy inputs and several
filters per batch, every image and probe compared bit-for-bit with the oracle. Inputs the
reference cannot take (the oracle rejects them: e.g. an index over 4096 entries or a
block over one page) must be rejected by the engine as well."""
import numpy as np
import pytest

from splinterdb_amd import engine as E

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N_CASES = 150


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def _case(rng):
    fp = int(rng.integers(18, 33))
    lis = int(rng.integers(3, 11)) if rng.random() < 0.85 else int(rng.integers(11, 13))
    cap = min(2 * 4096 * (1 << lis) - 1, (1 << fp) - 1)
    nf = int(rng.integers(1, 4))
    sizes = [max(1, int(np.exp(rng.uniform(0, np.log(cap / 2))))) for _ in range(nf)]
    vmax = min(63, (1 << (32 - fp)) - 1)
    vals = [int(rng.integers(0, vmax + 1)) for _ in range(nf)]
    dup = bool(rng.random() < 0.25)
    incr = bool(rng.random() < 0.4)
    return fp, lis, sizes, vals, dup, incr


def _hashes(rng, n, dup):
    h = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    if dup and n > 8:
        h = h[rng.integers(0, max(1, n // 8), size=n)]
    return h


def _oracle_add(oracle, ocfg, h, v, old=None):
    try:
        return oracle.filter_add(ocfg, h, value=v, old=old)
    except ValueError:
        return None


@pytest.mark.parametrize("seed", range(N_CASES))
def test_random_geometry_parity(oracle, seed):
    rng = np.random.default_rng(1000 + seed)
    fp, lis, sizes, vals, dup, incr = _case(rng)
    cfg = E.routing_config_init(fingerprint_size=fp, log_index_size=lis)
    ocfg = oracle.make_config(fingerprint_size=fp, log_index_size=lis)
    hs = [_hashes(rng, n, dup) for n in sizes]
    ofs = [_oracle_add(oracle, ocfg, h, v) for h, v in zip(hs, vals)]
    try:
        b = E.FilterBatch(cfg, sizes, vals)
    except E.PlatformStatusError:
        assert any(o is None for o in ofs), "engine rejected a batch the oracle accepts"
        return
    b.build_hashes(dev(np.concatenate(hs)))
    for f, of in enumerate(ofs):
        if of is None:
            with pytest.raises(E.PlatformStatusError):
                b.image(f)
            continue
        img = b.image(f)
        assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages), (seed, f)
        assert (img.pages == of.pages()).all(), (seed, f)
        assert (img.slots == of.slots()[: of.num_indices]).all(), (seed, f)
    # probes: each filter's own hashes plus random ones, routed at random
    good = [f for f, of in enumerate(ofs) if of is not None]
    if not good:
        return
    P = 20000
    ph = np.concatenate([np.concatenate(hs)[rng.integers(0, sum(sizes), size=P // 2)],
                         rng.integers(0, 1 << 32, size=P - P // 2, dtype=np.uint64).astype(np.uint32)])
    fid = np.array(good, dtype=np.uint32)[rng.integers(0, len(good), size=P)]
    found = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b.probe_hashes(dev(ph), dev(fid), P, found)
    torch.cuda.synchronize()
    got = found.cpu().numpy().view(np.uint64)
    for f in good:
        m = fid == f
        assert (got[m] == ofs[f].lookup_hashes(ph[m])).all(), (seed, f)
    # incremental add over filter `good[0]` with a value at least as wide
    if incr:
        f0 = good[0]
        n2 = max(1, sizes[f0] // 2)
        v2 = int(rng.integers(vals[f0], min(63, (1 << (32 - fp)) - 1) + 1))
        h2 = _hashes(rng, n2, dup)
        of2 = _oracle_add(oracle, ocfg, h2, v2, old=ofs[f0])
        try:
            b2 = E.FilterBatch(cfg, [n2], [v2], old=[(b, f0)])
            b2.build_hashes(dev(h2))
            img2 = b2.image(0)
        except E.PlatformStatusError:
            assert of2 is None, (seed, "engine rejected an incremental add the oracle accepts")
            return
        assert of2 is not None, (seed, "oracle rejected an incremental add the engine accepts")
        assert (img2.num_unique, img2.num_pages) == (of2.num_unique, of2.num_pages), seed
        assert (img2.pages == of2.pages()).all(), seed
        assert (img2.slots == of2.slots()[: of2.num_indices]).all(), seed


# Load factor ~1 (num_fingerprints within 2.6 % above a power of two, >= 2^13): the engine
# plans coarse buckets of 2^13 filter buckets with K4 bins of two buckets (FilterPlan.binsh).
# These geometries, fresh and incremental (32- and 64-bit pipelines), against the oracle.
@pytest.mark.parametrize("lis,fp,k", [(4, 22, 13), (6, 26, 16), (8, 26, 18), (8, 26, 20), (9, 30, 17),
                                      (11, 32, 19), (8, 32, 16)])
def test_load_factor_one_geometries(oracle, lis, fp, k):
    rng = np.random.default_rng(lis * 1000 + fp * 10 + k)
    cfg = E.routing_config_init(fingerprint_size=fp, log_index_size=lis)
    ocfg = oracle.make_config(fingerprint_size=fp, log_index_size=lis)
    vmax = min(63, (1 << (32 - fp)) - 1)
    sizes = [1 << k, (1 << k) + 5, int((1 << k) * 1.02)]
    vals = [int(rng.integers(0, vmax + 1)) for _ in sizes]
    hs = [_hashes(rng, n, dup=(i == 2)) for i, n in enumerate(sizes)]
    ofs = [oracle.filter_add(ocfg, h, value=v) for h, v in zip(hs, vals)]
    b = E.FilterBatch(cfg, sizes, vals)
    b.build_hashes(dev(np.concatenate(hs)))
    for f, of in enumerate(ofs):
        img = b.image(f)
        assert (img.num_unique, img.num_pages) == (of.num_unique, of.num_pages), f
        assert (img.pages == of.pages()).all(), f
        assert (img.slots == of.slots()[: of.num_indices]).all(), f
    # an incremental add whose total lands at load factor ~1 again: 2^(k+1) fingerprints
    n2 = (1 << (k + 1)) - sizes[0]
    v2 = vmax
    h2 = _hashes(rng, n2, dup=False)
    of2 = oracle.filter_add(ocfg, h2, value=v2, old=ofs[0])
    b2 = E.FilterBatch(cfg, [n2], [v2], old=[(b, 0)])
    b2.build_hashes(dev(h2))
    img2 = b2.image(0)
    assert (img2.num_unique, img2.num_pages) == (of2.num_unique, of2.num_pages)
    assert (img2.pages == of2.pages()).all()
    assert (img2.slots == of2.slots()[: of2.num_indices]).all()
    P = 20000
    allh = np.concatenate([h2, hs[0]])
    ph = np.concatenate([allh[rng.integers(0, allh.size, P // 2)],
                         rng.integers(0, 1 << 32, size=P - P // 2, dtype=np.uint64).astype(np.uint32)])
    found = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b2.probe_hashes(dev(ph), dev(np.zeros(P, dtype=np.uint32)), P, found)
    torch.cuda.synchronize()
    assert (found.cpu().numpy().view(np.uint64) == of2.lookup_hashes(ph)).all()


# Incremental adds whose new fingerprints pile into a few coarse buckets: the fused partition
# of the new keys spills (its fixed regions overflow), the fallback re-partitions them, and
# coarse buckets of new + old entries beyond LDS go to K4b -- both entry pipelines.
@pytest.mark.parametrize("entries", ["flag32", "wide64"])
def test_incremental_spill_and_big_buckets(oracle, entries, monkeypatch):
    if entries == "wide64":
        monkeypatch.setenv("RF_AMD_WIDE64", "1")
    rng = np.random.default_rng(77)
    cfg = E.routing_config_init(fingerprint_size=26, log_index_size=8)
    ocfg = oracle.make_config(fingerprint_size=26, log_index_size=8)
    h1 = rng.integers(0, 1 << 32, size=300_000, dtype=np.uint64).astype(np.uint32)
    of1 = oracle.filter_add(ocfg, h1, value=0)
    b1 = E.FilterBatch(cfg, [h1.size], [0])
    b1.build_hashes(dev(h1))
    # 32K new hashes: 12K copies of 5 values near one another (one coarse bucket: over its
    # SORT_CAP region and over LDS), the rest random
    hot = (np.uint32(0x9E370000) + np.arange(5, dtype=np.uint32) * np.uint32(97))
    h2 = np.concatenate([hot[rng.integers(0, 5, size=12_000)],
                         rng.integers(0, 1 << 32, size=20_000, dtype=np.uint64).astype(np.uint32)])
    rng.shuffle(h2)
    of2 = oracle.filter_add(ocfg, h2, value=1, old=of1)
    b2 = E.FilterBatch(cfg, [h2.size], [1], old=[(b1, 0)])
    b2.build_hashes(dev(h2))
    img = b2.image(0)
    assert (img.num_unique, img.num_pages) == (of2.num_unique, of2.num_pages)
    assert (img.pages == of2.pages()).all()
    assert (img.slots == of2.slots()[: of2.num_indices]).all()
    P = 20000
    ph = np.concatenate([h2[:P // 2], h1[:P // 2]])
    found = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b2.probe_hashes(dev(ph), dev(np.zeros(P, dtype=np.uint32)), P, found)
    torch.cuda.synchronize()
    assert (found.cpu().numpy().view(np.uint64) == of2.lookup_hashes(ph)).all()


@pytest.mark.parametrize("lis,n_old,frac_new,overlap", [(5, 33825, 0.5, 0.0), (5, 33825, 0.5, 0.3),
                                                        (8, 300000, 0.125, 0.2), (8, 300000, 0.4, 0.05),
                                                        (3, 6000, 0.33, 0.5), (8, 1 << 20, 0.33, 0.1)])
def test_incremental_new_entries_equal_to_old(oracle, lis, n_old, frac_new, overlap):
    """Incremental adds whose new hashes repeat old ones (same value: equal entries). The
    reference drops duplicates only among the new entries (src/routing_filter.c:559-597): a new
    entry equal to an old one is kept after it. Coarse buckets with new-entry counts on both
    sides of K4m's 2,048 (fuzz case 24 had one at exactly 2,048)."""
    rng = np.random.default_rng(lis * 1000 + n_old)
    fp, value = 26, 23
    cfg = E.routing_config_init(fingerprint_size=fp, log_index_size=lis)
    ocfg = oracle.make_config(fingerprint_size=fp, log_index_size=lis)
    h1 = rng.integers(0, 1 << 32, size=n_old, dtype=np.uint64).astype(np.uint32)
    n2 = int(n_old * frac_new)
    h2 = rng.integers(0, 1 << 32, size=n2, dtype=np.uint64).astype(np.uint32)
    k = int(n2 * overlap)
    h2[:k] = h1[rng.integers(0, n_old, size=k)]
    h2 = h2[rng.permutation(n2)]
    of = _oracle_add(oracle, ocfg, h1, value)
    of2 = _oracle_add(oracle, ocfg, h2, value, old=of)
    b = E.FilterBatch(cfg, [n_old], [value])
    b.build_hashes(dev(h1))
    b2 = E.FilterBatch(cfg, [n2], [value], old=[(b, 0)])
    b2.build_hashes(dev(h2))
    img = b2.image(0)
    assert (img.num_unique, img.num_pages) == (of2.num_unique, of2.num_pages)
    assert (img.slots == of2.slots()[: of2.num_indices]).all()
    assert (img.pages == of2.pages()).all()
