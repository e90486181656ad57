"""A/B of the incremental K4 variants in ONE process (diagnostics): the compaction chain's
round 8 (64 filters x 2^20-1 new keys onto 7 rounds of old entries, bench.py --workload
compaction) rebuilt repeatedly from the same round-7 batch with RF_AMD_K4_DIRECT = 0 (merge
path) and 1 (direct placement), interleaved; medians of the per-stage HIP event times; the
images of both must be identical.
usage: python tools/k4_ab.py [filters] [reps]"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n, V = (1 << 20) - 1, 8
dev = torch.device("cuda", 0)
cfg = E.routing_config_init(fingerprint_size=26, log_index_size=8, seed=42)
eng = E.Engine(0)
gid = torch.arange(F, device=dev, dtype=torch.int64)[:, None] << 32
j = torch.arange(n, device=dev, dtype=torch.int64)[None, :]
keys = [K.ids_keys_torch((gid + (v + 1) * j).reshape(-1), 24) for v in range(V)]
prev = None
for v in range(V - 1):
    b = E.FilterBatch(cfg, [n] * F, [v] * F, old=[(prev, f) for f in range(F)] if prev else None, engine=eng)
    b.build_keys(keys[v], 24)
    torch.cuda.synchronize()
    if prev is not None:
        prev.close()
    prev = b

modes = ["0", "1"]
res = {m: {} for m in modes}
digest = {}
for rnd in range(reps + 1):
    for m in modes:
        os.environ["RF_AMD_K4_DIRECT"] = m
        b = E.FilterBatch(cfg, [n] * F, [V - 1] * F, old=[(prev, f) for f in range(F)], engine=eng)
        b.set_timing(True)
        b.build_keys(keys[V - 1], 24)
        torch.cuda.synchronize()
        t = b.timings(0)
        if rnd > 0:
            for k, x in t.items():
                res[m].setdefault(k, []).append(x)
        if rnd == 0:
            h = hashlib.sha256()
            for f in (0, 1, F - 1):
                img = b.image(f)
                h.update(img.pages.tobytes())
                h.update(img.slots.tobytes())
            h.update(np.array([i.num_unique for i in b.infos()], dtype=np.uint64).tobytes())
            digest[m] = h.hexdigest()
        b.close()
out = {m: {k: round(float(np.median(x)), 4) for k, x in r.items() if k != "probe"} for m, r in res.items()}
print(json.dumps({"filters": F, "keys_per_round": n, "round": V, "stages_ms": out,
                  "identical": digest["0"] == digest["1"]}))
if digest["0"] != digest["1"]:
    raise SystemExit("K4 variants differ")
