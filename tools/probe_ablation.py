"""Diagnostic: time k_probe truncated after each step (hash / + probe-line load / full),
interleaved rounds in one process (cdna_hip_programming.md rule 24).
usage: python tools/probe_ablation.py [filters=8] [keys_per_filter=8000000]  (C3: 256 1048576)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8_000_000
N = F * n
cfg = E.routing_config_init()
dev = torch.device("cuda", 0)
keys = K.seq_keys_torch(0, N, 24, dev)
fid = (torch.arange(N, device=dev) // n).to(torch.int32)
found = torch.empty(N, dtype=torch.int64, device=dev)
b = E.FilterBatch(cfg, [n] * F)
b.set_timing(True)
b.build_keys(keys, 24)
torch.cuda.synchronize()
L = E.load_library()
res = {m: [] for m in (1, 2, 0)}
for rnd in range(6):
    for m in (1, 2, 0):
        L.rf_amd_debug_probe_ablate(m)
        b.probe_keys(keys, 24, fid, N, found)
        torch.cuda.synchronize()
        res[m].append(b.timings()["probe"])
L.rf_amd_debug_probe_ablate(0)
out = {("hash", "line", "full")[i]: round(float(np.median(res[m][1:])), 4)
       for i, m in enumerate((1, 2, 0))}
print(json.dumps(out))
