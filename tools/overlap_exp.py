"""Experiment: does a probe of one batch overlap a build of another on MI355X?
Serialized: build(k) -> probe(k) on one stream. Double-buffered: builds on stream A, probes
on stream B, batch k % 2, with events so build(k+2) waits for probe(k)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

F, n = 8, 8_000_000
N = F * n
cfg = E.routing_config_init()
dev = torch.device("cuda", 0)
keys = K.seq_keys_torch(0, N, 24, dev)
fid = (torch.arange(N, device=dev, dtype=torch.int64) // n).to(torch.int32)
found = [torch.empty(N, dtype=torch.int64, device=dev) for _ in range(2)]
bs = [E.FilterBatch(cfg, [n] * F) for _ in range(2)]
counts = [n] * F
lo_p, hi_p = torch.cuda.Stream.priority_range()
PRI = os.environ.get("OVL_PRI", "")  # "build" / "probe": that stream gets the high priority
sA = torch.cuda.Stream(priority=hi_p if PRI == "build" else lo_p)
sB = torch.cuda.Stream(priority=hi_p if PRI == "probe" else lo_p)
steps = 20


def serial():
    for k in range(steps):
        b = bs[k % 2]
        b.build_keys(keys, 24, stream=sA.cuda_stream)
        b.probe_keys_runs(keys, 24, counts, found[k % 2], stream=sA.cuda_stream)


def overlapped():
    built = [torch.cuda.Event() for _ in range(steps)]
    probed = [torch.cuda.Event() for _ in range(steps)]
    for k in range(steps):
        b = bs[k % 2]
        if k >= 2:
            sA.wait_event(probed[k - 2])
        b.build_keys(keys, 24, stream=sA.cuda_stream)
        built[k].record(sA)
        sB.wait_event(built[k])
        b.probe_keys_runs(keys, 24, counts, found[k % 2], stream=sB.cuda_stream)
        probed[k].record(sB)


for name, fn in (("serial", serial), ("overlapped", overlapped), ("serial", serial), ("overlapped", overlapped)):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ok = all(bool(((f & 1) == 1).all().item()) for f in found)
    print(f"[{PRI or 'equal'}] {name:10s} {dt * 1e3:.3f} ms/step  {N / dt / 1e6:,.0f} Mkeys/s  ok={ok}")
