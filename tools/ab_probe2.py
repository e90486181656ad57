"""A/B of librf_amd builds in ONE process, interleaved rounds: probe (and build) kernel
times at C2 (8 x 8M, probes grouped by filter) and C3 (256 x 2^20), plus result identity.
usage: python tools/ab_probe2.py libA.so libB.so ...   (prints one JSON line)"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

vp = ctypes.c_void_p
dev = torch.device("cuda", 0)
cfg = E.RfConfig(26, 8, 42, 4096, 32)
shapes = {"c2": (8, 8_000_000), "c3": (256, 1 << 20)}
if os.environ.get("AB_SHAPES"):  # e.g. AB_SHAPES=c3: one shape per process (PMC passes)
    shapes = {k: shapes[k] for k in os.environ["AB_SHAPES"].split(",")}
out = {}
for shape, (F, n) in shapes.items():
    N = F * n
    keys = K.seq_keys_torch(0, N, 24, dev)
    counts = (ctypes.c_uint64 * F)(*([n] * F))
    libs = []
    for arg in sys.argv[1:]:
        # path[:VAR=V,VAR2=V2] -- environment set around this entry's calls
        path, _, sw = arg.partition(":")
        L = ctypes.CDLL(os.path.abspath(path))
        L.rf_amd_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        L.rf_amd_batch_create.argtypes = [vp, ctypes.POINTER(E.RfConfig), ctypes.c_uint32, vp, vp, vp, vp,
                                          ctypes.POINTER(vp)]
        L.rf_amd_batch_build_keys.argtypes = [vp, vp, ctypes.c_uint32, vp]
        L.rf_amd_batch_probe_keys_runs.argtypes = [vp, vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), vp, vp]
        L.rf_amd_batch_set_timing.argtypes = [vp, ctypes.c_int]
        L.rf_amd_batch_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.c_uint32]
        L.rf_amd_batch_destroy.argtypes = [vp]
        e = vp()
        assert L.rf_amd_engine_create(0, ctypes.byref(e)) == 0
        nn = np.full(F, n, dtype=np.uint32)
        vals = np.zeros(F, dtype=np.uint16)
        b = vp()
        assert L.rf_amd_batch_create(e, ctypes.byref(cfg), F, nn.ctypes.data, vals.ctypes.data, None, None,
                                     ctypes.byref(b)) == 0
        assert L.rf_amd_batch_set_timing(b, 1) == 0
        found = torch.empty(N, dtype=torch.int64, device=dev)
        libs.append((os.path.basename(os.path.dirname(path)) + "/" + os.path.basename(path) + (":" + sw if sw else ""),
                     L, b, found, nn, vals, sw))
    torch.cuda.synchronize()
    res = {name: {"probe": [], "build": [], "assemble": [], "sort": [], "partition": [], "layout": []} for name, *_ in libs}
    arr = (ctypes.c_float * 9)()
    for rnd in range(7):
        for name, L, b, found, nn_, vals_, sw in libs:
            saved = {}
            for kv in (sw.split(",") if sw else []):  # this entry's switches, restored after it
                k_, _, v_ = kv.partition("=")
                saved[k_] = os.environ.get(k_)
                os.environ[k_] = v_
            assert L.rf_amd_batch_build_keys(b, keys.data_ptr(), 24, None) == 0
            assert L.rf_amd_batch_probe_keys_runs(b, keys.data_ptr(), 24, counts, found.data_ptr(), None) == 0
            torch.cuda.synchronize()
            for k_, v_ in saved.items():
                if v_ is None:
                    os.environ.pop(k_, None)
                else:
                    os.environ[k_] = v_
            L.rf_amd_batch_timings(b, arr, 9)
            r = res[name]
            r["probe"].append(arr[8]); r["build"].append(arr[7]); r["assemble"].append(arr[6])
            r["sort"].append(arr[3]); r["partition"].append(arr[0]); r["layout"].append(arr[5])
    ref = libs[0][3]
    same = all(torch.equal(ref, x[3]) for x in libs[1:])
    allfound = bool(((ref & 1) == 1).all())
    diff = {}
    for name, _, _, fo, *_ in libs[1:]:
        bad = torch.nonzero(ref != fo).flatten()
        if bad.numel():
            sel = bad[:12]
            diff[name] = {"count": int(bad.numel()), "idx": sel.tolist(), "want": ref[sel].tolist(),
                          "got": fo[sel].tolist(), "lanes_in_wave": (sel % 64).tolist()}
    out[shape] = {"identical": same, "all_found": allfound, "diff": diff,
                  **{k: {m: round(float(np.median(v[m][1:])), 4) for m in v} for k, v in res.items()}}
    for name, L, b, *_ in libs:
        L.rf_amd_batch_destroy(b)
    del keys, libs
    torch.cuda.empty_cache()
print(json.dumps(out))
