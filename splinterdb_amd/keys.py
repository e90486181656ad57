"""Synthetic key sets for the routing-filter workloads.

* sequential-id keys in the reference's filter_test format
  (tests/functional/filter_test.c:172-183): little-endian u64 id in bytes 0-7, zeros after;
* random fixed-length keys: bytes from splitmix64(seed 0x5EED);
* variable-length keys, lengths uniform in [8, 100] (seeded), bytes from splitmix64.

numpy versions are the host generators; the torch versions build the same bytes directly
in device memory so bench inputs never cross PCIe.
"""
import numpy as np

GOLDEN_GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """Element i = splitmix64 output number (start + i) for the given seed."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(start, start + n, dtype=np.uint64) + np.uint64(1)) * GOLDEN_GAMMA
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def seq_keys(start: int, n: int, key_len: int = 24) -> np.ndarray:
    k = np.zeros((n, key_len), dtype=np.uint8)
    ids = np.arange(start, start + n, dtype=np.uint64)
    k[:, :8] = ids.view(np.uint8).reshape(n, 8)
    return k


def ids_keys(ids, key_len: int = 24) -> np.ndarray:
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    k = np.zeros((ids.size, key_len), dtype=np.uint8)
    k[:, :8] = ids.view(np.uint8).reshape(ids.size, 8)
    return k


def random_keys(n: int, key_len: int = 24, seed: int = 0x5EED, start: int = 0) -> np.ndarray:
    words = (key_len + 7) // 8
    r = splitmix64(seed, n * words, start * words)
    return r.view(np.uint8).reshape(n, words * 8)[:, :key_len].copy()


def var_keys(n: int, lo: int = 8, hi: int = 100, seed: int = 0x5EED):
    """Returns (bytes u8[total], offsets u64[n+1])."""
    lens = (splitmix64(seed ^ 0x1E57, n) % np.uint64(hi - lo + 1)).astype(np.int64) + lo
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    total = int(offs[-1])
    data = splitmix64(seed, (total + 7) // 8).view(np.uint8)[:total].copy()
    return data, offs


# ---- device-side generators (torch, for bench inputs resident in HBM) ----------------
def seq_keys_torch(start: int, n: int, key_len: int, device):
    import torch
    k = torch.zeros((n, key_len), dtype=torch.uint8, device=device)
    ids = torch.arange(start, start + n, dtype=torch.int64, device=device)
    k[:, :8] = ids.view(torch.uint8).view(n, 8)
    return k


def ids_keys_torch(ids, key_len: int = 24):
    """filter_test-format keys of the given ids (int64 device tensor), on its device."""
    import torch
    n = ids.numel()
    k = torch.zeros((n, key_len), dtype=torch.uint8, device=ids.device)
    k[:, :8] = ids.contiguous().view(torch.uint8).view(n, 8)
    return k


# ---- C5: variable-length keys + Zipf(0.99) probe mix -----------------
def zipf_ids(n: int, count: int, s: float = 0.99, seed: int = 1) -> np.ndarray:
    """`count` ids in [0, n) with P(rank r) ~ r^-s (rank 1 hottest); ranks are scattered
    over the ids by an odd multiplier so hot keys are not adjacent."""
    rng = np.random.default_rng(seed)
    cdf = np.cumsum(np.arange(1, n + 1, dtype=np.float64) ** -s)
    cdf /= cdf[-1]
    r = np.minimum(np.searchsorted(cdf, rng.random(count), side="right"), n - 1)
    return (r.astype(np.uint64) * np.uint64(2654435761)) % np.uint64(n)


def gather_var(data: np.ndarray, offs: np.ndarray, ids: np.ndarray, chunk: int = 1 << 20):
    """Variable-length keys `ids` of (data, offs) as a new (bytes, offsets) pair."""
    ids = np.asarray(ids, dtype=np.int64)
    lens = (offs[ids + 1] - offs[ids]).astype(np.int64)
    po = np.zeros(ids.size + 1, dtype=np.uint64)
    np.cumsum(lens, out=po[1:])
    out = np.empty(int(po[-1]), dtype=np.uint8)
    for c0 in range(0, ids.size, chunk):
        c1 = min(ids.size, c0 + chunk)
        b0, b1 = int(po[c0]), int(po[c1])
        src = offs[ids[c0:c1]].astype(np.int64) - po[c0:c1].astype(np.int64)
        idx = np.repeat(src, lens[c0:c1]) + np.arange(b0, b1, dtype=np.int64)
        out[b0:b1] = data[idx]
    return out, po


def c5_inputs(num_filters: int, keys_per_filter: int, seed: int = 0x5EED, pos_frac: float = 0.9):
    """C5 per GPU: num_filters filters of variable-length (8-100 B) keys, and as many probes
    as keys: pos_frac positives drawn Zipf(0.99) within each filter (probing that filter),
    the rest uniform negatives routed to random filters, all shuffled together.
    Returns dict(bytes, offs, probe_bytes, probe_offs, probe_fid, positive)."""
    n = num_filters * keys_per_filter
    data, offs = var_keys(n, seed=seed)
    npos = int(keys_per_filter * pos_frac)
    ids = np.concatenate([f * keys_per_filter + zipf_ids(keys_per_filter, npos, seed=seed + f).astype(np.int64)
                          for f in range(num_filters)])
    pos_fid = np.repeat(np.arange(num_filters, dtype=np.uint32), npos)
    nneg = n - ids.size
    neg_d, neg_o = var_keys(nneg, seed=seed ^ 0xBADD)
    rng = np.random.default_rng(seed)
    neg_fid = rng.integers(0, num_filters, size=nneg, dtype=np.uint32)
    # one shuffled probe stream: gather positives from the key set, negatives from their own
    allb = np.concatenate([data, neg_d])
    allo = np.concatenate([offs[:-1], neg_o + offs[-1]])
    src = np.concatenate([ids, np.arange(n, n + nneg, dtype=np.int64)])
    fid = np.concatenate([pos_fid, neg_fid])
    positive = np.concatenate([np.ones(ids.size, bool), np.zeros(nneg, bool)])
    perm = rng.permutation(src.size)
    pb, po = gather_var(allb, allo, src[perm])
    return dict(bytes=data, offs=offs, probe_bytes=pb, probe_offs=po, probe_fid=fid[perm],
                positive=positive[perm])
