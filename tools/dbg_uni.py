"""Diagnostics: probe C2 (8 x 8M keys, per-filter runs) with the given library and dump, for
the first mismatching probes of filter 0, the hash, bucket and probe line (JSON)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

F, n = 8, 8_000_000
dev = torch.device("cuda", 0)
cfg = E.routing_config_init(26, 8, 42)
keys = K.seq_keys_torch(0, F * n, 24, dev)
b = E.FilterBatch(cfg, [n] * F)
b.build_keys(keys, 24)
found = torch.empty(F * n, dtype=torch.int64, device=dev)
out = {}
for rep in range(3):
    b.probe_keys_runs(keys, 24, [n] * F, found)
    torch.cuda.synchronize()
    bad = torch.nonzero((found & 1) == 0).flatten()
    out[f"rep{rep}_bad"] = int(bad.numel())
    out[f"rep{rep}_first"] = bad[:8].tolist()
bad0 = bad[bad < n][:16].cpu().numpy()
h = torch.empty(F * n, dtype=torch.int32, device=dev)
E.hash_keys(cfg, keys, 24, F * n, h)
hh = h.cpu().numpy().view(np.uint32)
lines = b.debug_lines()
inf = b.info(0)
rows = []
for i in bad0:
    rows.append({"i": int(i), "hash": int(hh[i]), "found": int(found[i].item())})
out["rows"] = rows
out["num_lines"] = int(lines.shape[0])
out["info0"] = [inf.num_fingerprints, inf.num_unique, inf.num_pages, inf.num_indices]
# lines of filter 0 only: first num_lines / F (same geometry for every filter)
np.save("gpurun_out/dbg_lines0.npy", lines[: lines.shape[0] // F])
# and the hash-only found values via the hash path (per-probe filter ids)
fid = torch.zeros(n, dtype=torch.int32, device=dev)
f2 = torch.empty(n, dtype=torch.int64, device=dev)
b.probe_hashes(h[:n], fid, n, f2)
torch.cuda.synchronize()
out["hash_path_bad"] = int(((f2 & 1) == 0).sum().item())
print(json.dumps(out))
