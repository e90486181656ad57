"""k_probe's fast path (full waves of one filter, plan in scalar registers, lines in LDS in
natural order) against the oracle's routing_filter_lookup (src/routing_filter.c:985-1073):
every probe's found_values equal, for 24-byte keys and for hashes, with run bounds that do and
do not fall on wave boundaries, a misaligned key buffer (general path), values 0-63 (SWAR
compare with value bits) and overflowed probe lines (image walk from the fast path); and at
C2's filter size, the fast path equal to the general path (per-probe filter ids)."""
import numpy as np
import pytest

from splinterdb_amd import engine as E
from splinterdb_amd import keys as K

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")



def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def build(oracle, cfg_kw, sizes, vals, seed):
    cfg = E.routing_config_init(**cfg_kw)
    ocfg = oracle.make_config(**cfg_kw)
    keys = K.random_keys(sum(sizes), seed=seed)
    b = E.FilterBatch(cfg, sizes, vals)
    b.build_keys(dev(keys), 24)
    hashes = oracle.hash_fixed(keys.reshape(-1), 24)
    ofs, s = [], 0
    for n, v in zip(sizes, vals):
        ofs.append(oracle.filter_add(ocfg, hashes[s:s + n], value=v))
        s += n
    return b, keys, hashes, ofs


def probe_set(rng, keys, hashes, sizes, counts):
    """counts[f] probes of filter f: half its own keys, half random keys"""
    pk, starts = [], np.concatenate([[0], np.cumsum(sizes)])
    for f, c in enumerate(counts):
        k = K.random_keys(c, seed=int(rng.integers(1 << 30)))
        own = c // 2
        if own:
            k[:own] = keys[starts[f] + rng.integers(0, sizes[f], size=own)]
        pk.append(k)
    return np.concatenate(pk)


@pytest.mark.parametrize("seed", [3, 10])
def test_fast_path_vs_oracle(oracle, seed):
    rng = np.random.default_rng(seed)
    sizes = [300000, 70000, 1 << 17, 5000, 200001]
    vals = [0, 5, 63, 1, 31]
    b, keys, hashes, ofs = build(oracle, {"log_index_size": 8}, sizes, vals, seed=42)
    for counts in ([64 * 3000, 64 * 700, 64 * 2000, 64 * 50, 64 * 2500],     # on wave boundaries
                   [191999, 44444, 130001, 3333, 160000 + 7]):               # not
        pk = probe_set(rng, keys, hashes, sizes, counts)
        ph = oracle.hash_fixed(pk.reshape(-1), 24)
        want = np.concatenate([ofs[f].lookup_hashes(ph[sum(counts[:f]):sum(counts[:f + 1])])
                               for f in range(len(sizes))])
        N = len(pk)
        for how in ("keys", "hashes", "keys_misaligned"):
            found = torch.zeros(N, dtype=torch.int64, device="cuda:0")
            if how == "keys":
                b.probe_keys_runs(dev(pk), 24, counts, found)
            elif how == "hashes":
                b.probe_hashes_runs(dev(ph), counts, found)
            else:  # 8 bytes into a buffer: the general path (16-byte LDS-DMA needs alignment)
                buf = torch.zeros(N * 24 + 16, dtype=torch.uint8, device="cuda:0")
                buf[8:8 + N * 24] = dev(pk.reshape(-1).view(np.uint8))
                b.probe_keys_runs(buf[8:], 24, counts, found)
            torch.cuda.synchronize()
            got = found.cpu().numpy().view(np.uint64)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (how, seed, bad.size, bad[:8].tolist(), got[bad[:4]], want[bad[:4]])


def test_fast_path_overflowed_lines_walk_the_image(oracle):
    """clustered fingerprints overflow probe lines: the fast path's walk of the image"""
    rng = np.random.default_rng(11)
    fps, lis, n, value = 26, 8, 400000, 3
    cfg_kw = {"fingerprint_size": fps, "log_index_size": lis}
    lnb = max(int(n).bit_length() - 1, lis)
    rem, sh = fps - lnb, 32 - fps
    h = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    k = 0
    for c in range(16):
        b0 = int(rng.integers(0, (1 << lnb) - 4))
        for j in range(150):
            fp = ((b0 + j % 4) << rem) | (j * 7919 % (1 << rem))
            h[k] = np.uint32((fp << sh) | (j & ((1 << sh) - 1)))
            k += 1
    b = E.FilterBatch(E.routing_config_init(**cfg_kw), [n], [value])
    b.build_hashes(dev(h))
    of = oracle.filter_add(oracle.make_config(**cfg_kw), h, value=value)
    P = 64 * 5000
    ph = rng.integers(0, 1 << 32, size=P, dtype=np.uint64).astype(np.uint32)
    ph[: P // 3] = h[rng.integers(0, n, size=P // 3)]
    ph[P // 3: P // 3 + k] = h[:k]
    ph[P // 3 + k: P // 3 + 2 * k] = h[:k] ^ np.uint32(1 << sh)
    found = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b.probe_hashes_runs(dev(ph), [P], found)
    torch.cuda.synchronize()
    got = found.cpu().numpy().view(np.uint64)
    want = of.lookup_hashes(ph)
    assert (got == want).all(), int((got != want).sum())
    assert (got[: P // 3] >> np.uint64(value) & np.uint64(1)).all()


def test_fast_path_equals_general_path_at_c2_size():
    """an 8M-key filter (C2's per-filter size) probed through the fast path (runs) and the
    general path (per-probe filter ids): identical results, every key found"""
    cfg = E.routing_config_init(log_index_size=8)
    n = 8_000_000
    keys = K.seq_keys_torch(0, n, 24, torch.device("cuda", 0))
    b = E.FilterBatch(cfg, [n], [7])
    b.build_keys(keys, 24)
    f_fast = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    b.probe_keys_runs(keys, 24, [n], f_fast)
    f_gen = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    b.probe_keys(keys, 24, torch.zeros(n, dtype=torch.int32, device="cuda:0"), n, f_gen)
    torch.cuda.synchronize()
    assert bool(((f_fast >> 7) & 1).all())
    assert torch.equal(f_fast, f_gen)


def test_probe_floor_stays_in_bounds():
    """rf_amd_debug_probe_floor (bench.py's measured floor) over runs that do and do not fall on
    wave boundaries: it writes exactly the n output words, nothing past them"""
    cfg = E.routing_config_init(log_index_size=8)
    sizes = [300000, 5000, 200001]
    keys = K.seq_keys_torch(0, sum(sizes), 24, torch.device("cuda", 0))
    b = E.FilterBatch(cfg, sizes, [0, 1, 2])
    b.build_keys(keys, 24)
    for counts in ([64 * 3000, 64 * 50, 64 * 2500], [191999, 3333, 160007]):
        N = sum(counts)
        out = torch.full((N + 4096,), -7, dtype=torch.int64, device="cuda:0")
        b.probe_floor(keys, 24, counts, out)
        h = torch.zeros(N, dtype=torch.int32, device="cuda:0")
        E.hash_keys(cfg, keys[:N], 24, N, h)
        b.probe_floor(h, 4, counts, out)
        torch.cuda.synchronize()
        assert bool((out[N:] == -7).all())
        assert int((out[:N] == -7).sum()) == 0
    with pytest.raises(Exception):
        b.probe_floor(keys, 8, [1, 1, 1], out)
