"""Diagnostic: k_probe at capped occupancy (waves/SIMD via LDS padding), interleaved."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

F, n = 8, 8_000_000
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
ref = None
modes = [8, 6, 5, 4, 3, 2]
res = {m: [] for m in modes}
for rnd in range(6):
    for m in modes:
        L.rf_amd_debug_probe_ablate(m << 8)
        b.probe_keys(keys, 24, fid, N, found)
        torch.cuda.synchronize()
        res[m].append(b.timings()["probe"])
        if ref is None:
            ref = found.clone()
        else:
            assert torch.equal(ref, found)
L.rf_amd_debug_probe_ablate(0)
print(json.dumps({f"occ{m}": round(float(np.median(v[1:])), 4) for m, v in res.items()}))
