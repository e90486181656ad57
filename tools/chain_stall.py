"""Host-side stall finder for the compaction chain (bench.py --workload compaction): the same
rounds, each host call timed; prints every call over AB_STALL_MS (50) and per-call maxima.
env: AB_F (64), AB_N (1048575), AB_STEPS (30)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

dev = torch.device("cuda", 0)
F = int(os.environ.get("AB_F", 64))
n = int(os.environ.get("AB_N", (1 << 20) - 1))
STEPS = int(os.environ.get("AB_STEPS", 30))
LIM = float(os.environ.get("AB_STALL_MS", 50))
V = 8
cfg = E.routing_config_init(fingerprint_size=26, log_index_size=8, seed=42)
eng = E.Engine(0)
stream = torch.cuda.Stream(device=dev)
st = stream.cuda_stream
with torch.cuda.stream(stream):
    gid = torch.arange(F, device=dev, dtype=torch.int64)[:, None] << 32
    j = torch.arange(n, device=dev, dtype=torch.int64)[None, :]
    keys = [K.ids_keys_torch((gid + (v + 1) * j).reshape(-1), 24) for v in range(V)]
stream.synchronize()
mx = {}


def tick(name, t0, step, v):
    dt = (time.perf_counter() - t0) * 1e3
    mx[name] = max(mx.get(name, 0.0), dt)
    if dt > LIM:
        print(f"step {step} round {v} {name} {dt:.1f} ms", flush=True)
    return time.perf_counter()


for step in range(STEPS):
    prev = None
    for v in range(V):
        t = time.perf_counter()
        b = E.FilterBatch(cfg, [n] * F, [v] * F, old=[(prev, f) for f in range(F)] if prev else None, engine=eng)
        t = tick("create", t, step, v)
        b.build_keys(keys[v], 24, stream=st)
        t = tick("build", t, step, v)
        if prev is not None:
            prev.close(stream=st)
        t = tick("close", t, step, v)
        b.infos(stream=st)
        t = tick("infos", t, step, v)
        prev = b
    stream.synchronize()
    prev.close(stream=st)
    stream.synchronize()
    fr, tot = torch.cuda.mem_get_info(dev)
    print(f"step {step} pool {eng.pool_stats()} device free {fr / 2**30:.2f} GiB of {tot / 2**30:.1f}", flush=True)
print({k: round(x, 2) for k, x in mx.items()}, flush=True)
