"""What the per-stage HIP events cost the C2 step: the same build + probe timed with every
stage event, with the probe's two events only, and with no events, interleaved in one
process (reps rounds of `steps` steps each). Prints one JSON line."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402


def main():
    F, n, steps, reps = 8, 8_000_000, 20, 5
    dev = torch.device("cuda", 0)
    cfg = E.routing_config_init(fingerprint_size=26, log_index_size=8, seed=42)
    eng = E.Engine(0)
    stream = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(stream):
        keys = K.seq_keys_torch(0, F * n, 24, dev)
        found = torch.empty(F * n, dtype=torch.int64, device=dev)
    stream.synchronize()
    batch = E.FilterBatch(cfg, [n] * F, engine=eng)
    counts = [n] * F

    def step():
        batch.build_keys(keys, 24, stream=stream.cuda_stream)
        batch.probe_keys_runs(keys, 24, counts, found, stream=stream.cuda_stream)

    modes = {"all": dict(enable=True, sets=steps), "probe": dict(enable=True, sets=steps, probe_only=True),
             "none": dict(enable=False)}
    res = {m: [] for m in modes}
    stage = {m: [] for m in modes}
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for _ in range(reps):
        for m, kw in modes.items():
            batch.set_timing(**kw)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            res[m].append((time.perf_counter() - t0) / steps * 1e3)
            if kw.get("enable"):
                t = [batch.timings(b) for b in range(steps)]
                stage[m].append({k: round(statistics.median(x[k] for x in t), 4) for k in ("build_total", "probe")})
    print(json.dumps({"ms_per_step": {m: [round(x, 4) for x in v] for m, v in res.items()},
                      "median": {m: round(statistics.median(v), 4) for m, v in res.items()},
                      "event_stages": stage}))


if __name__ == "__main__":
    main()
