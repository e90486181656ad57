"""Diagnostic: C2 probe under several rf_amd_debug_probe_ablate words (bits 8-15 waves/SIMD
cap, bits 16-23 probes per lane), interleaved rounds in ONE process, results checked equal.
usage: python tools/probe_variants.py ppl:occ [ppl:occ ...]   e.g. 1:8 2:8 3:8"""
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
modes = [tuple(int(x) for x in m.split(":")) for m in (sys.argv[1:] or ["1:8", "2:8"])]
res = {m: [] for m in modes}
ref = None
for rnd in range(7):
    for m in modes:
        L.rf_amd_debug_probe_ablate((m[0] << 16) | (m[1] << 8))
        b.probe_keys(keys, 24, fid, N, found)
        torch.cuda.synchronize()
        res[m].append(b.timings()["probe"])
        if ref is None:
            ref = found.clone()
        else:
            assert torch.equal(ref, found), m
L.rf_amd_debug_probe_ablate(0)
b.probe_keys(keys, 24, fid, N, found)
torch.cuda.synchronize()
assert torch.equal(ref, found)
print(json.dumps({f"ppl{m[0]}_occ{m[1]}": round(float(np.median(v[1:])), 4) for m, v in res.items()}))
