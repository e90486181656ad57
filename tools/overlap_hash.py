"""Experiment: split the probe into its key hashing (independent of the build) and its line
gathers, and hash the probe keys on a second stream while the build runs. C2 shape, one
process; prints ms/step per variant (median of reps) as one JSON line.
  fused      build_keys + probe_keys_runs on one stream (the bench's step)
  split      build_keys; hash_keys; probe_hashes_runs on one stream
  ovl_lo/hi  hash_keys on a second stream (low / high priority) started with the build;
             probe_hashes_runs waits for it
"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402


def main():
    F, n, steps, reps = 8, 8_000_000, 20, 5
    N = F * n
    dev = torch.device("cuda", 0)
    cfg = E.routing_config_init(fingerprint_size=26, log_index_size=8, seed=42)
    eng = E.Engine(0)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    sA = torch.cuda.Stream(device=dev, priority=hi)
    sL = torch.cuda.Stream(device=dev, priority=lo)
    sH = torch.cuda.Stream(device=dev, priority=hi)
    keys = K.seq_keys_torch(0, N, 24, dev)
    found = torch.empty(N, dtype=torch.int64, device=dev)
    hashes = torch.empty(N, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    b = E.FilterBatch(cfg, [n] * F, engine=eng)
    counts = [n] * F

    def fused():
        b.build_keys(keys, 24, stream=sA.cuda_stream)
        b.probe_keys_runs(keys, 24, counts, found, stream=sA.cuda_stream)

    def split():
        b.build_keys(keys, 24, stream=sA.cuda_stream)
        E.hash_keys(cfg, keys, 24, N, hashes, stream=sA.cuda_stream, engine=eng)
        b.probe_hashes_runs(hashes, counts, found, stream=sA.cuda_stream)

    def ovl(sh):
        def f():
            e0 = torch.cuda.Event()
            e0.record(sA)  # the previous step's probe has read the hashes
            sh.wait_event(e0)
            E.hash_keys(cfg, keys, 24, N, hashes, stream=sh.cuda_stream, engine=eng)
            e1 = torch.cuda.Event()
            e1.record(sh)
            b.build_keys(keys, 24, stream=sA.cuda_stream)
            sA.wait_event(e1)
            b.probe_hashes_runs(hashes, counts, found, stream=sA.cuda_stream)
        return f

    variants = {"fused": fused, "split": split, "ovl_lo": ovl(sL), "ovl_hi": ovl(sH)}
    res = {k: [] for k in variants}
    for f in variants.values():
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    ok = {}
    for _ in range(reps):
        for k, f in variants.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                f()
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / steps * 1e3)
            ok[k] = bool(((found & 1) == 1).all().item())
            found.zero_()
    print(json.dumps({"priority_range": [lo, hi], "median_ms": {k: round(statistics.median(v), 4) for k, v in res.items()},
                      "ms": {k: [round(x, 4) for x in v] for k, v in res.items()}, "all_found": ok}))


if __name__ == "__main__":
    main()
