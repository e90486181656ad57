"""Diagnostics: only the callback-driven async lookups of tools/shim_latency.py (8,192 states
over 8 filters, 64 in flight, as tests/functional/test_async.c drives them), shim and
reference stacks, median of AD_REPS (7) runs; prints one JSON line. Set RF_SHIM_SUBMIT_PROFILE=1
/ RF_AMD_SUBMIT_PROFILE=1 for the per-step submit cycles (stderr, at exit)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import refimpl as R  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

REPS = int(os.environ.get("AD_REPS", 7))
n = (1 << 20) - 1
out = {}
for name, path in (("shim", R.SHIM_PATH), ("reference", R.LIB_PATH)):
    if os.environ.get("AD_ONLY") and os.environ["AD_ONLY"] != name:
        continue
    with R.Stack(path=path, cache_mib=4096, disk_mib=16384) as s:
        keys = [K.ids_keys((np.uint64(f) << np.uint64(32)) + np.arange(n, dtype=np.uint64)) for f in range(8)]
        descs = [s.add(s.hash_keys(k), value=i % 8) for i, k in enumerate(keys)]
        rng = np.random.default_rng(1)
        P = 8192
        fid = rng.integers(0, 8, size=P).astype(np.uint32)
        probe = np.stack([keys[f][rng.integers(0, n)] for f in fid])
        s.lookup_keys_async_driven(descs, probe, fid, max_inflight=64)
        ab0 = s.async_breakdown()
        ts = []
        for _ in range(REPS):
            t = time.perf_counter()
            s.lookup_keys_async_driven(descs, probe, fid, max_inflight=64)
            ts.append(time.perf_counter() - t)
        ab1 = s.async_breakdown()
        r = {"async_driven_8192_ms": round(float(np.median(ts)) * 1e3, 3),
             "min_ms": round(min(ts) * 1e3, 3)}
        if ab0:
            d = {k: ab1[k] - ab0[k] for k in ab0}
            nb = max(d["batches"], 1)
            r["breakdown"] = {
                "reaps_per_run": round(d["batches"] / REPS, 1), "states_per_reap": round(d["states"] / nb, 1),
                "submit_us_per_state": round(d["submit_ns"] / max(d["states"], 1) / 1e3, 3),
                "reap_us_per_reap": round(d["reap_ns"] / nb / 1e3, 2),
                "callbacks_us_per_reap": round(d["callback_ns"] / nb / 1e3, 2)}
        out[name] = r
print(json.dumps(out), flush=True)
