"""A/B: the C2 probe with two builds of librf_amd in ONE process, interleaved rounds
(cdna_hip_programming.md rule 24). usage: python tools/ab_probe.py libA.so libB.so ..."""
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
N = F * n
dev = torch.device("cuda", 0)
keys = K.seq_keys_torch(0, N, 24, dev)
fid = (torch.arange(N, device=dev) // n).to(torch.int32)
outs = {}
vp = ctypes.c_void_p
cfg = E.RfConfig(26, 8, 42, 4096, 32)
libs = []
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    L.rf_amd_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.rf_amd_batch_create.argtypes = [vp, ctypes.POINTER(E.RfConfig), ctypes.c_uint32, vp, vp, vp, vp, ctypes.POINTER(vp)]
    L.rf_amd_batch_build_keys.argtypes = [vp, vp, ctypes.c_uint32, vp]
    L.rf_amd_batch_probe_keys.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_uint64, vp, vp]
    L.rf_amd_batch_set_timing.argtypes = [vp, ctypes.c_int]
    L.rf_amd_batch_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.c_uint32]
    e = vp(); assert L.rf_amd_engine_create(0, ctypes.byref(e)) == 0
    nn = np.full(F, n, dtype=np.uint32); vals = np.zeros(F, dtype=np.uint16)
    b = vp(); assert L.rf_amd_batch_create(e, ctypes.byref(cfg), F, nn.ctypes.data, vals.ctypes.data, None, None, ctypes.byref(b)) == 0
    assert L.rf_amd_batch_set_timing(b, 1) == 0
    assert L.rf_amd_batch_build_keys(b, keys.data_ptr(), 24, None) == 0
    found = torch.empty(N, dtype=torch.int64, device=dev)
    libs.append((os.path.basename(path), L, b, found, nn, vals))
torch.cuda.synchronize()
res = {name: {"probe": [], "build": []} for name, *_ in libs}
arr = (ctypes.c_float * 9)()
for rnd in range(8):
    for name, L, b, found, *_ in libs:
        assert L.rf_amd_batch_build_keys(b, keys.data_ptr(), 24, None) == 0
        assert L.rf_amd_batch_probe_keys(b, keys.data_ptr(), 24, fid.data_ptr(), N, found.data_ptr(), None) == 0
        torch.cuda.synchronize()
        L.rf_amd_batch_timings(b, arr, 9)
        res[name]["probe"].append(arr[8]); res[name]["build"].append(arr[7])
ref = libs[0][3]
same = all(torch.equal(ref, x[3]) for x in libs[1:])
print(json.dumps({"identical_results": same, **{k: {m: round(float(np.median(v[m][1:])), 4) for m in v} for k, v in res.items()}}))
