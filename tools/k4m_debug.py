"""Diagnostic (not a test): fuzz case 24's incremental add (fp 26, lis 5, 33,825 old + 16,912 new
hashes, value 23) built by the engine and by the oracle; prints where the images differ (first
differing slots / page bytes, and the coarse bucket of the index) -- RF_AMD_K4M=0/1 decides
which bucket sort the engine uses."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splinterdb_amd import engine as E  # noqa: E402
from oracle import oracle as O  # noqa: E402

d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "k4m_case24.npz"))
h1, h2 = d["h1"], d["h2"]
fp, lis = 26, 5
cfg = E.routing_config_init(fingerprint_size=fp, log_index_size=lis)
ocfg = O.make_config(fingerprint_size=fp, log_index_size=lis)
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")  # noqa: E731
b = E.FilterBatch(cfg, [len(h1)], [23])
b.build_hashes(dev(h1))
b2 = E.FilterBatch(cfg, [len(h2)], [23], old=[(b, 0)])
b2.build_hashes(dev(h2))
img = b2.image(0)
of = O.filter_add(ocfg, h1, value=23)
of2 = O.filter_add(ocfg, h2, value=23, old=of)
print("K4M", os.environ.get("RF_AMD_K4M", "1"), "unique", img.num_unique, of2.num_unique, "pages", img.num_pages,
      of2.num_pages)
os_ = of2.slots()[: of2.num_indices]
ds = np.flatnonzero(img.slots != os_)
print("slots differ:", ds.size, "first", ds[:8].tolist(), "cb(128 idx)", sorted(set((ds // 128).tolist()))[:16])
if ds.size:
    i = ds[0]
    print("  slot", i, "engine", [hex(x) for x in img.slots[max(0, i - 2):i + 3]], "oracle",
          [hex(x) for x in os_[max(0, i - 2):i + 3]])
op = of2.pages()
db = np.flatnonzero(img.pages != op)
print("page bytes differ:", db.size, "first", db[:8].tolist())
if db.size:
    j = db[0]
    # the index whose block holds byte j: the last slot at or before it
    print("  engine", img.pages[j - 8:j + 24].tolist())
    print("  oracle", op[j - 8:j + 24].tolist())
    print("  slots around:", [(k, hex(int(s))) for k, s in enumerate(os_) if abs(int(s) - int(j)) < 2048][:6])
