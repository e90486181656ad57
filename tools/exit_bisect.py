"""Diagnostic (not a test): which part of tools/shim_latency.py leaves the process to die at
exit ("munmap_chunk(): invalid pointer"). usage: python tools/exit_bisect.py MODE
MODE: 0 shim stack only; 1 + adds; 2 + lookups; 3 + async many; 4 + async driven;
5 + mt chains; 6 the reference stack with everything; 7 the shim stack with everything, then
the reference stack with everything (one process, as shim_latency.py); 8 the same, each step 6x;
9 the shim stack: 512 filters of 2,000 keys, async lookups over all of them"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import refimpl as R  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

mode = int(sys.argv[1])
n = (1 << 20) - 1


def run(path, top, reps=1):
    with R.Stack(path=path, cache_mib=16384, disk_mib=131072) as s:
        if top >= 1:
            keys = [K.ids_keys((np.uint64(f) << np.uint64(32)) + np.arange(n, dtype=np.uint64)) for f in range(8)]
            hs = [s.hash_keys(k) for k in keys]
            base = s.add(hs[0])
            for _ in range(reps):
                s.add(hs[0])
                s.add(hs[1], value=1, old=base)
            descs = [s.add(h, value=i % 8) for i, h in enumerate(hs)]
            rng = np.random.default_rng(1)
            fid = rng.integers(0, 8, size=8192).astype(np.uint32)
            probe = np.stack([keys[f][rng.integers(0, n)] for f in fid])
        for _ in range(reps):
            if top >= 2:
                s.lookup_keys(descs[0], probe[:2000])
                s.lookup_batch(descs, probe, fid)
            if top >= 3:
                s.lookup_keys_async_many(descs, probe, fid)
            if top >= 4:
                s.lookup_keys_async_driven(descs, probe, fid, max_inflight=64)
        if top >= 5:
            mkeys = K.ids_keys(np.arange(8 * n, dtype=np.uint64) + np.uint64(1 << 40))
            pr = K.random_keys(8 * 16, seed=1)
            for _ in range(min(reps, 3)):
                s.mt_chains(mkeys, 8, 1, n, pr, 16)


if mode == 9:
    with R.Stack(path=R.SHIM_PATH, cache_mib=16384, disk_mib=131072) as s:
        many = [s.add(s.hash_keys(K.ids_keys((np.uint64(100 + f) << np.uint64(32)) +
                                             np.arange(2000, dtype=np.uint64))), value=f % 30)
                for f in range(512)]
        probe = K.random_keys(8192, seed=3)
        fid512 = np.random.default_rng(2).integers(0, 512, size=8192).astype(np.uint32)
        for _ in range(6):
            s.lookup_keys_async_many(many, probe, fid512)
elif mode <= 5:
    run(R.SHIM_PATH, mode)
elif mode == 6:
    run(R.LIB_PATH, 5)
else:
    run(R.SHIM_PATH, 5, reps=1 if mode == 7 else 6)
    run(R.LIB_PATH, 5, reps=1 if mode == 7 else 6)
print("mode", mode, "done", flush=True)
