"""A/B diagnostic: build the same 8M-key filter with two librf_amd builds and report the
first differing index slot / page byte."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402

vp = ctypes.c_void_p
n = int(os.environ.get("AB_N", "8000000"))
keys = K.seq_keys_torch(0, n, 24, torch.device("cuda", 0))
cfg = E.RfConfig(26, 8, 42, 4096, 32)
imgs = []
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    L.rf_amd_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.rf_amd_batch_create.argtypes = [vp, ctypes.POINTER(E.RfConfig), ctypes.c_uint32, vp, vp, vp, vp, ctypes.POINTER(vp)]
    L.rf_amd_batch_build_keys.argtypes = [vp, vp, ctypes.c_uint32, vp]
    L.rf_amd_batch_info.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(E.RfFilterInfo)]
    L.rf_amd_batch_read_image.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint64, vp, ctypes.c_uint32]
    e = vp(); assert L.rf_amd_engine_create(0, ctypes.byref(e)) == 0
    nn = np.array([n], dtype=np.uint32); vals = np.zeros(1, dtype=np.uint16)
    b = vp(); assert L.rf_amd_batch_create(e, ctypes.byref(cfg), 1, nn.ctypes.data, vals.ctypes.data, None, None, ctypes.byref(b)) == 0
    assert L.rf_amd_batch_build_keys(b, keys.data_ptr(), 24, None) == 0
    inf = E.RfFilterInfo(); assert L.rf_amd_batch_info(b, 0, ctypes.byref(inf)) == 0
    pages = np.zeros(inf.num_pages * 4096, dtype=np.uint8); slots = np.zeros(inf.num_indices, dtype=np.uint64)
    rc = L.rf_amd_batch_read_image(b, 0, pages.ctypes.data, pages.size, slots.ctypes.data, slots.size)
    imgs.append((path, inf.num_unique, inf.num_pages, inf.error, pages, slots))
    print(path, "unique", inf.num_unique, "pages", inf.num_pages, "err", inf.error, "rc", rc)
(_, _, _, _, pa, sa), (_, _, _, _, pb, sb) = imgs[0], imgs[1]
d = np.nonzero(sa != sb)[0]
print("slot diffs", d.size, "first", d[:5])
if d.size:
    i = int(d[0])
    for j in range(max(0, i - 2), min(sa.size, i + 3)):
        ca = int(pa[int(sa[j])]) | (int(pa[int(sa[j]) + 1]) << 8)
        cb = int(pb[int(sb[j])]) | (int(pb[int(sb[j]) + 1]) << 8) if int(sb[j]) + 1 < pb.size else -1
        print(j, "A", int(sa[j]), divmod(int(sa[j]), 4096), ca, "B", int(sb[j]), divmod(int(sb[j]), 4096), cb)
