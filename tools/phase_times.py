"""Per-phase shader-clock timing of the instrumented build kernels (diagnostics).
Run on the GPU box: python tools/phase_times.py [kid] [filters] [keys_per_filter]
(PT_CHAIN=R: stamp round R of compaction chains instead of a fresh build)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import build as B  # noqa: E402

os.environ["RF_AMD_LIB"] = os.environ.get("PT_LIB") or B.LIB_STAMPS  # stamps: diagnostics build only
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

KID = int(sys.argv[1]) if len(sys.argv) > 1 else 1  # 1 = bucket sort, 2 = fused partition
F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
n = int(sys.argv[3]) if len(sys.argv) > 3 else 8_000_000
cfg = E.routing_config_init()
CHAIN = int(os.environ.get("PT_CHAIN", "0"))  # > 0: stamp round CHAIN of compaction chains
buf = torch.zeros(1 << 24, dtype=torch.int64, device="cuda:0")
L = E.load_library()
if CHAIN:
    # bench.py --workload compaction's chains: round v of filter g adds (g << 32) + (v + 1) j
    gid = torch.arange(F, device="cuda:0", dtype=torch.int64)[:, None] << 32
    j = torch.arange(n, device="cuda:0", dtype=torch.int64)[None, :]
    prev = None
    for v in range(CHAIN):
        keys = K.ids_keys_torch((gid + (v + 1) * j).reshape(-1), 24)
        b = E.FilterBatch(cfg, [n] * F, [v] * F, old=[(prev, f) for f in range(F)] if prev else None)
        if v == CHAIN - 1:
            torch.cuda.synchronize()
            E._check(L.rf_amd_debug_phase_buffer(buf.data_ptr(), KID))
        b.build_keys(keys, 24)
        torch.cuda.synchronize()
        prev = b
else:
    keys = K.seq_keys_torch(0, F * n, 24, "cuda:0")
    b = E.FilterBatch(cfg, [n] * F)
    for _ in range(2):
        b.build_keys(keys, 24)
    torch.cuda.synchronize()
    E._check(L.rf_amd_debug_phase_buffer(buf.data_ptr(), KID))
    b.build_keys(keys, 24)
    torch.cuda.synchronize()
E._check(L.rf_amd_debug_phase_buffer(None, 0))
ts = buf.cpu().numpy().reshape(-1, 16)
used = ts[:, 8] != 0
ts = ts[used]
print(f"workgroups stamped: {ts.shape[0]}")
if KID == 1:
    names = {15: "entry", 0: "init", 1: "load+rank", 2: "bin scan", 3: "scatter", 4: "bin sort",
             9: "merge split (t0)", 10: "merge run (t0)", 5: "scan+compact", 6: "write out",
             7: "index bounds", 8: "uniq+end"}
    order = [15, 0, 1, 2, 3, 4, 9, 10, 5, 6, 7, 8]
elif KID == 5:
    names = {15: "entry", 0: "new load", 1: "rank+DMA issue", 2: "bin scan", 3: "scatter", 4: "bin sort+old landed",
             5: "dedupe+compact", 6: "merge (split + run)", 7: "index bounds", 8: "uniq+end"}
    order = [15, 0, 1, 2, 3, 4, 5, 6, 7, 8]
elif KID == 4:
    names = {15: "entry", 5: "size loads (t0)", 6: "scan", 0: "excl store", 1: "next()", 2: "doubling",
             3: "pages+slots", 8: "quirk+end"}
    order = [15, 5, 6, 0, 1, 2, 3, 8]
elif KID == 3:
    names = {15: "entry", 0: "metadata", 1: "fill", 2: "entry runs", 3: "store", 4: "line scan",
             8: "line write"}
    order = [15, 0, 1, 2, 3, 4, 8]
else:
    names = {15: "entry", 0: "init", 5: "load+hash (thread 0)", 1: "rank", 2: "scan+reserve",
             3: "stage", 4: "slots", 8: "write runs"}
    order = [15, 0, 5, 1, 2, 3, 4, 8]
tot = (ts[:, 8] - ts[:, 15]).astype(np.float64)
print(f"per workgroup: mean {tot.mean():.0f} cycles, median {np.median(tot):.0f}")
for a, c in zip(order[:-1], order[1:]):
    d = (ts[:, c] - ts[:, a]).astype(np.float64)
    print(f"  {names[c]:16s} {d.mean():9.0f} cycles  ({100 * d.mean() / tot.mean():5.1f} %)")
