"""Diagnostics: fixed costs of one host-buffer lookup round trip in the engine (no shim):
rf_amd_batch_probe_hashes_host on one filter and rf_amd_probe_many_hashes_host over 8
single-filter batches, for 1 / 1,024 / 8,192 hashes. Prints one JSON line (ms, median)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402

L = E.load_library()
cfg = E.routing_config_init()
eng = E.Engine(0)
rng = np.random.default_rng(0)
batches = []
for f in range(8):
    h = rng.integers(0, 1 << 32, size=1 << 20, dtype=np.uint64).astype(np.uint32)
    b = E.FilterBatch(cfg, [h.size], engine=eng)
    E._check(L.rf_amd_batch_build_hashes_host(b.h, h.ctypes.data))
    batches.append(b)


def med(fn, reps=20):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return round(float(np.median(ts)) * 1e3, 4)


out = {}
for n in (1, 16, 1024, 8192):
    q = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    found = np.zeros(n, dtype=np.uint64)
    out[f"one_filter_{n}"] = med(lambda: E._check(L.rf_amd_batch_probe_hashes_host(
        batches[0].h, q.ctypes.data, None, n, found.ctypes.data)))
    counts = np.full(8, n // 8 if n >= 8 else 0, dtype=np.uint64)
    counts[0] += n - counts.sum()
    arr = (ctypes.c_void_p * 8)(*[b.h.value for b in batches])
    out[f"eight_filters_{n}"] = med(lambda: E._check(L.rf_amd_probe_many_hashes_host(
        eng.h, arr, None, counts.ctypes.data, 8, q.ctypes.data, found.ctypes.data)))
print(json.dumps(out))
