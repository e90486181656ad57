"""A/B of the probe kernels in ONE process (diagnostics): k_probe (one 64-probe tile per wave)
against k_probe_pipe (persistent waves, next tile's keys fetched while this tile's lines are
in flight; RF_AMD_PROBE_PIPE = workgroups per CU), at C2 (8 x 8,000,000) and C3 (256 x 2^20),
interleaved rounds, medians of the probe's HIP event time; results must be identical.
usage: python tools/probe_pipe_ab.py [c2|c3] [pipe values ...]   e.g. c2 0 7 8 4"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "c2"
modes = sys.argv[2:] or ["0", "7"]
F, n = (8, 8_000_000) if w == "c2" else (256, 1 << 20)
N = F * n
cfg = E.routing_config_init()
dev = torch.device("cuda", 0)
keys = K.seq_keys_torch(0, N, 24, dev)
found = torch.empty(N, dtype=torch.int64, device=dev)
b = E.FilterBatch(cfg, [n] * F)
b.set_timing(True)
b.build_keys(keys, 24)
torch.cuda.synchronize()
counts = [n] * F
res = {m: [] for m in modes}
ref = None
for rnd in range(9):
    for m in modes:
        os.environ["RF_AMD_PROBE_PIPE"] = m
        b.probe_keys_runs(keys, 24, counts, found)
        torch.cuda.synchronize()
        if rnd > 0:
            res[m].append(b.timings()["probe"])
        if ref is None:
            ref = found.clone()
        elif not torch.equal(found, ref):
            raise SystemExit(f"mode {m}: results differ")
out = {m: round(float(np.median(v)), 4) for m, v in res.items()}
print(json.dumps({"workload": w, "probe_ms": out, "all_found": bool(((ref & 1) == 1).all().item())}))
