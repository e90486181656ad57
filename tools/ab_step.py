"""A/B of librf_amd builds in ONE process: the C2 bench step (build + probe runs of 8 x 8M
24-B keys) timed with no HIP events, interleaved rounds, medians; results checked equal.
usage: python tools/ab_step.py libA.so libB.so ...   (prints one JSON line)"""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

vp = ctypes.c_void_p
dev = torch.device("cuda", 0)
cfg = E.RfConfig(26, 8, 42, 4096, 32)
F, n, steps, rounds = 8, 8_000_000, 20, 7
N = F * n
keys = K.seq_keys_torch(0, N, 24, dev)
counts = (ctypes.c_uint64 * F)(*([n] * F))
stream = torch.cuda.Stream(device=dev)
libs = []
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    L.rf_amd_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.rf_amd_batch_create.argtypes = [vp, ctypes.POINTER(E.RfConfig), ctypes.c_uint32, vp, vp, vp, vp, ctypes.POINTER(vp)]
    L.rf_amd_batch_build_keys.argtypes = [vp, vp, ctypes.c_uint32, vp]
    L.rf_amd_batch_probe_keys_runs.argtypes = [vp, vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), vp, vp]
    e = vp()
    assert L.rf_amd_engine_create(0, ctypes.byref(e)) == 0
    nn = np.full(F, n, dtype=np.uint32)
    vals = np.zeros(F, dtype=np.uint16)
    b = vp()
    assert L.rf_amd_batch_create(e, ctypes.byref(cfg), F, nn.ctypes.data, vals.ctypes.data, None, None, ctypes.byref(b)) == 0
    found = torch.empty(N, dtype=torch.int64, device=dev)
    libs.append((os.path.basename(path), L, b, found, nn, vals))
st = vp(stream.cuda_stream)


def step(L, b, found):
    assert L.rf_amd_batch_build_keys(b, keys.data_ptr(), 24, st) == 0
    assert L.rf_amd_batch_probe_keys_runs(b, keys.data_ptr(), 24, counts, found.data_ptr(), st) == 0


res = {name: [] for name, *_ in libs}
for name, L, b, found, *_ in libs:
    for _ in range(3):
        step(L, b, found)
torch.cuda.synchronize()
for _ in range(rounds):
    for name, L, b, found, *_ in libs:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(L, b, found)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / steps * 1e3)
ref = libs[0][3]
same = all(torch.equal(ref, x[3]) for x in libs[1:])
print(json.dumps({"identical": same, "all_found": bool(((ref & 1) == 1).all()),
                  "ms_per_step_median": {k: round(statistics.median(v), 4) for k, v in res.items()},
                  "ms": {k: [round(x, 4) for x in v] for k, v in res.items()}}))
