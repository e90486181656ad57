"""Diagnostic: probe-line group size (RF_AMD_LINE_SIGMA, read at batch creation) x probe
occupancy (waves/SIMD), C2 probe timed with HIP events, interleaved rounds in ONE process.
usage: python tools/line_sigma.py [sigma ...]"""
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
sigmas = [float(x) for x in sys.argv[1:]] or [5.0, 4.0, 3.0, 2.0]
occs = [0, 8, 5, 4]  # 0 = production (6 waves/SIMD)
L = E.load_library()
batches = {}
for sg in sigmas:
    os.environ["RF_AMD_LINE_SIGMA"] = str(sg)
    b = E.FilterBatch(cfg, [n] * F)
    b.set_timing(True)
    b.build_keys(keys, 24)
    batches[sg] = b
os.environ.pop("RF_AMD_LINE_SIGMA")
torch.cuda.synchronize()
ref = None
res = {(sg, o): [] for sg in sigmas for o in occs}
build = {sg: [] for sg in sigmas}
for rnd in range(6):
    for sg, b in batches.items():
        L.rf_amd_debug_probe_ablate(0)
        b.build_keys(keys, 24)
        torch.cuda.synchronize()
        build[sg].append(b.timings()["build_total"])
        for o in occs:
            L.rf_amd_debug_probe_ablate(o << 8)
            b.probe_keys(keys, 24, fid, N, found)
            torch.cuda.synchronize()
            res[(sg, o)].append(b.timings()["probe"])
            if ref is None:
                ref = found.clone()
            else:
                assert torch.equal(ref, found), (sg, o)
L.rf_amd_debug_probe_ablate(0)
print(json.dumps({"build": {str(sg): round(float(np.median(v[1:])), 4) for sg, v in build.items()},
                  "probe": {f"sigma{sg}_occ{o}": round(float(np.median(v[1:])), 4) for (sg, o), v in res.items()}}))
