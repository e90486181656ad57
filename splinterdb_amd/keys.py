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
