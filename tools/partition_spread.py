"""Diagnostics: is the fused partition's run-to-run spread tied to buffer placement?
Builds C2 with several batches (separate device allocations) and several key buffers in
one process and prints the partition stage time of each combination."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

F, n = 8, 8_000_000
cfg = E.routing_config_init()
keysets = [K.seq_keys_torch(0, F * n, 24, "cuda:0") for _ in range(2)]
batches = [E.FilterBatch(cfg, [n] * F) for _ in range(3)]
for b in batches:
    b.set_timing(True, sets=8)
for ki, keys in enumerate(keysets):
    for bi, b in enumerate(batches):
        for _ in range(8):
            b.build_keys(keys, 24)
        torch.cuda.synchronize()
        part = [b.timings(back)["partition"] for back in range(8)]
        print(f"keys {ki} batch {bi}: partition {np.mean(part):.4f} ms (min {np.min(part):.4f}, max {np.max(part):.4f})",
              flush=True)
