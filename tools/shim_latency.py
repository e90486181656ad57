"""Diagnostics: the drop-in shim's per-call costs on the GPU box, beside the reference's
own routing_filter.c in the same page stack (oracle/_ref/libshim_rf.so vs libref_rf.so).
Prints one JSON line: routing_filter_add of 2^20 hashes (fresh, onto an old filter),
routing_filter_lookup of one key, routing_filter_amd_lookup_batch of 8,192 (filter, key)
pairs over 8 filters, and 8,192 routing_filter_lookup_async states."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import refimpl as R  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402


def med(f, reps=5):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return round(float(np.median(ts)) * 1e3, 3)


out = {}
n = (1 << 20) - 1
for name, path in (("shim", R.SHIM_PATH), ("reference", R.LIB_PATH)):
    with R.Stack(path=path, cache_mib=8192, disk_mib=65536) as s:
        keys = [K.ids_keys((np.uint64(f) << np.uint64(32)) + np.arange(n, dtype=np.uint64)) for f in range(8)]
        hs = [s.hash_keys(k) for k in keys]
        s.add(hs[0])  # warm
        r = {"add_fresh_ms": med(lambda: s.add(hs[0])),
             "add_incremental_ms": med(lambda: s.add(hs[1], value=1, old=s.add(hs[0])))}
        descs = [s.add(h, value=i % 8) for i, h in enumerate(hs)]
        rng = np.random.default_rng(1)
        P = 8192
        fid = rng.integers(0, 8, size=P).astype(np.uint32)
        probe = np.stack([keys[f][rng.integers(0, n)] for f in fid])
        r["lookup_one_ms"] = med(lambda: s.lookup_keys(descs[0], probe[:1]))
        r["lookup_batch_8192_ms"] = med(lambda: s.lookup_batch(descs, probe, fid))
        r["lookup_async_8192_ms"] = med(lambda: s.lookup_keys_async_many(descs, probe, fid))
        out[name] = r
print(json.dumps(out))
