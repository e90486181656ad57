"""Experiment: does the fused partition's time (C2: 8 x 8M 24-B keys) depend on where the key
array starts? The same keys are copied to a byte offset inside one large allocation; per
offset, the median partition stage time over interleaved rounds. Prints one JSON line."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

F, n = 8, 8_000_000
N = F * n
dev = torch.device("cuda", 0)
cfg = E.routing_config_init(fingerprint_size=26, log_index_size=8, seed=42)
keys = K.seq_keys_torch(0, N, 24, dev).view(-1)
offsets = [0, 64, 128, 256, 1024, 4096, 65536, 1 << 21]
big = torch.empty(keys.numel() + max(offsets) + 256, dtype=torch.uint8, device=dev)
b = E.FilterBatch(cfg, [n] * F)
b.set_timing(True)
res = {o: [] for o in offsets}
for rnd in range(5):
    for o in offsets:
        kv = big[o:o + keys.numel()]
        kv.copy_(keys)
        for _ in range(2):
            b.build_keys(kv, 24)
        torch.cuda.synchronize()
        t = []
        for _ in range(3):
            b.build_keys(kv, 24)
            torch.cuda.synchronize()
            t.append(b.timings()["partition"])
        res[o].append(statistics.median(t))
print(json.dumps({"base_mod_2M": big.data_ptr() % (1 << 21),
                  "partition_ms_median": {str(o): round(statistics.median(v), 4) for o, v in res.items()},
                  "partition_ms": {str(o): [round(x, 4) for x in v] for o, v in res.items()}}))
