"""A/B of librf_amd builds in ONE process: the C2 build (8 x 8M 24-B keys) with per-stage
HIP-event timing, interleaved rounds, per-stage medians; every library's filter images, slots
and probe results checked byte-equal to the first's.
usage: python tools/ab_build.py libA.so libB.so ...   (prints one JSON line)"""
import ctypes
import hashlib
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

vp = ctypes.c_void_p
dev = torch.device("cuda", 0)
cfg = E.RfConfig(26, 8, 42, 4096, 32)
F = int(os.environ.get("AB_F", "8"))
n = int(os.environ.get("AB_N", "8000000"))
steps, rounds = 10, 7
N = F * n
keys = K.seq_keys_torch(0, N, 24, dev)
counts = (ctypes.c_uint64 * F)(*([n] * F))
stream = torch.cuda.Stream(device=dev)
st = vp(stream.cuda_stream)
NS = len(E.FilterBatch.STAGES)
libs = []
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    L.rf_amd_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.rf_amd_batch_create.argtypes = [vp, ctypes.POINTER(E.RfConfig), ctypes.c_uint32, vp, vp, vp, vp, ctypes.POINTER(vp)]
    L.rf_amd_batch_build_keys.argtypes = [vp, vp, ctypes.c_uint32, vp]
    L.rf_amd_batch_probe_keys_runs.argtypes = [vp, vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), vp, vp]
    L.rf_amd_batch_set_timing.argtypes = [vp, ctypes.c_int]
    L.rf_amd_batch_timings_back.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_float), ctypes.c_uint32]
    L.rf_amd_batch_info.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(E.RfFilterInfo)]
    L.rf_amd_batch_read_image.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint64, vp, ctypes.c_uint32]
    e = vp()
    assert L.rf_amd_engine_create(0, ctypes.byref(e)) == 0
    nn = np.full(F, n, dtype=np.uint32)
    vals = np.zeros(F, dtype=np.uint16)
    b = vp()
    assert L.rf_amd_batch_create(e, ctypes.byref(cfg), F, nn.ctypes.data, vals.ctypes.data, None, None, ctypes.byref(b)) == 0
    assert L.rf_amd_batch_set_timing(b, steps) == 0
    found = torch.empty(N, dtype=torch.int64, device=dev)
    libs.append((os.path.basename(path), L, b, found))


def digest(L, b):
    h = hashlib.sha256()
    for f in range(F):
        inf = E.RfFilterInfo()
        assert L.rf_amd_batch_info(b, f, ctypes.byref(inf)) == 0 and inf.error == 0
        pages = np.zeros(inf.num_pages * cfg.page_size, dtype=np.uint8)
        slots = np.zeros(inf.num_indices, dtype=np.uint64)
        assert L.rf_amd_batch_read_image(b, f, pages.ctypes.data, pages.nbytes, slots.ctypes.data, inf.num_indices) == 0
        h.update(pages.tobytes())
        h.update(slots.tobytes())
        h.update(bytes(inf))
    return h.hexdigest()


res = {name: {s: [] for s in E.FilterBatch.STAGES} for name, *_ in libs}
for name, L, b, found in libs:
    for _ in range(2):
        assert L.rf_amd_batch_build_keys(b, keys.data_ptr(), 24, st) == 0
torch.cuda.synchronize()
for _ in range(rounds):
    for name, L, b, found in libs:
        for _ in range(steps):
            assert L.rf_amd_batch_build_keys(b, keys.data_ptr(), 24, st) == 0
        stream.synchronize()
        arr = (ctypes.c_float * NS)()
        for back in range(steps):
            assert L.rf_amd_batch_timings_back(b, back, arr, NS) == 0
            for s, v in zip(E.FilterBatch.STAGES, arr):
                res[name][s].append(float(v))
digests = {}
probe = os.environ.get("AB_NOPROBE") != "1"  # timing-only variants (wrong images): no probe
for name, L, b, found in libs:
    if probe:
        assert L.rf_amd_batch_probe_keys_runs(b, keys.data_ptr(), 24, counts, found.data_ptr(), st) == 0
    stream.synchronize()
    digests[name] = digest(L, b)
ref = libs[0][3]
print(json.dumps({"images_identical": len(set(digests.values())) == 1,
                  "probes_identical": probe and all(torch.equal(ref, x[3]) for x in libs[1:]),
                  "all_found": probe and bool(((ref & 1) == 1).all()),
                  "stage_ms_median": {k: {s: round(statistics.median(v), 4) for s, v in d.items() if s != "probe"}
                                      for k, d in res.items()}}))
