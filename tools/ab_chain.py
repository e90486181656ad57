"""A/B of librf_amd builds in ONE process on the compaction chain's incremental builds (bench.py
--workload compaction: F filters, each grown by R incremental adds of n keys; round v adds keys
(f << 32) + (v + 1) j with value v). Per library and repetition a whole chain is built; the
stage times (HIP events) of its last round are recorded, and the final images are compared
across libraries (SHA-256 of every filter's pages and slots).
usage: python tools/ab_chain.py lib1.so[:VAR=V,...] lib2.so ...   (one JSON line)
env: AB_F (64), AB_N (1048575), AB_R (8 rounds), AB_REPS (3)"""
import ctypes
import hashlib
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
F = int(os.environ.get("AB_F", 64))
n = int(os.environ.get("AB_N", (1 << 20) - 1))
R = int(os.environ.get("AB_R", 8))
REPS = int(os.environ.get("AB_REPS", 3))
cfg = E.RfConfig(26, 8, 42, 4096, 32)
STAGES = ["partition", "count_scan", "scatter", "cb_sort", "cb_sort_big", "layout", "assemble", "build_total"]

gid = torch.arange(F, device=dev, dtype=torch.int64)[:, None] << 32
jj = torch.arange(n, device=dev, dtype=torch.int64)[None, :]
round_keys = [K.ids_keys_torch((gid + (v + 1) * jj).reshape(-1), 24) for v in range(R)]

libs = []
for arg in sys.argv[1:]:
    path, _, envs = arg.partition(":")
    L = ctypes.CDLL(os.path.abspath(path))
    L.rf_amd_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.rf_amd_batch_create.argtypes = [vp, ctypes.POINTER(E.RfConfig), ctypes.c_uint32, vp, vp, vp, vp,
                                      ctypes.POINTER(vp)]
    L.rf_amd_batch_build_keys.argtypes = [vp, vp, ctypes.c_uint32, vp]
    L.rf_amd_batch_set_timing.argtypes = [vp, ctypes.c_int]
    L.rf_amd_batch_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.c_uint32]
    L.rf_amd_batch_destroy.argtypes = [vp]
    L.rf_amd_batch_info.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(E.RfFilterInfo)]
    L.rf_amd_batch_read_image.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint64, vp, ctypes.c_uint32]
    e = vp()
    assert L.rf_amd_engine_create(0, ctypes.byref(e)) == 0
    name = os.path.basename(os.path.dirname(path)) + "/" + os.path.basename(path) + (":" + envs if envs else "")
    libs.append((name, L, e, envs))


def chain(L, e):
    prev = None
    nn = np.full(F, n, dtype=np.uint32)
    arr = (ctypes.c_float * 9)()
    for v in range(R):
        vals = np.full(F, v, dtype=np.uint16)
        b = vp()
        if prev is None:
            assert L.rf_amd_batch_create(e, ctypes.byref(cfg), F, nn.ctypes.data, vals.ctypes.data, None, None,
                                         ctypes.byref(b)) == 0
        else:
            olds = (vp * F)(*([prev] * F))
            oidx = np.arange(F, dtype=np.uint32)
            assert L.rf_amd_batch_create(e, ctypes.byref(cfg), F, nn.ctypes.data, vals.ctypes.data, olds,
                                         oidx.ctypes.data, ctypes.byref(b)) == 0
        if v == R - 1:
            assert L.rf_amd_batch_set_timing(b, 1) == 0
        assert L.rf_amd_batch_build_keys(b, round_keys[v].data_ptr(), 24, None) == 0
        torch.cuda.synchronize()
        if prev is not None:
            L.rf_amd_batch_destroy(prev)
        prev = b
    L.rf_amd_batch_timings(prev, arr, 9)
    return prev, {s: float(arr[i]) for i, s in enumerate(STAGES)}


def digest(L, b):
    h = hashlib.sha256()
    info = E.RfFilterInfo()
    for f in range(F):
        assert L.rf_amd_batch_info(b, f, ctypes.byref(info)) == 0
        pages = np.zeros(info.num_pages * 4096, dtype=np.uint8)
        slots = np.zeros(info.num_indices, dtype=np.uint64)
        assert L.rf_amd_batch_read_image(b, f, pages.ctypes.data, pages.size, slots.ctypes.data, slots.size) == 0
        h.update(pages.tobytes())
        h.update(slots.tobytes())
        h.update(np.array([info.num_unique, info.num_pages], dtype=np.uint64).tobytes())
    return h.hexdigest()[:16]


res = {name: {s: [] for s in STAGES} for name, *_ in libs}
digests = {}
for rep in range(REPS):
    for name, L, e, envs in libs:
        saved = {}
        for kv in (envs.split(",") if envs else []):  # this entry's switches, restored after it
            k_, _, v_ = kv.partition("=")
            saved[k_] = os.environ.get(k_)
            os.environ[k_] = v_
        b, t = chain(L, e)
        for k_, v_ in saved.items():
            if v_ is None:
                os.environ.pop(k_, None)
            else:
                os.environ[k_] = v_
        for s in STAGES:
            res[name][s].append(t[s])
        if rep == 0:
            digests[name] = digest(L, b)
        L.rf_amd_batch_destroy(b)
out = {"filters": F, "keys_per_round": n, "round": R, "reps": REPS,
       "identical": len(set(digests.values())) == 1, "digests": digests,
       "stages_ms_median": {k: {s: round(float(np.median(v[s])), 4) for s in STAGES} for k, v in res.items()}}
print(json.dumps(out))
