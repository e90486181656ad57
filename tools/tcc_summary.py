"""Per-kernel L2 (TCC) summary from rocprofv3 --pmc counter_collection.csv files
(diagnostics): per-launch hits, misses, hit rate and HBM read requests, one table per file.
usage: python tools/tcc_summary.py <c2.csv> [<c3.csv> ...]"""
import collections
import csv
import os
import sys

sys.path.insert(0, "profiles")
from pmc_summary import short  # noqa: E402

for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        s = short(r["Kernel_Name"]) or r["Kernel_Name"].split("(")[0][:24]
        agg[s][r["Counter_Name"].replace("_sum", "")].append(float(r["Counter_Value"]))
    print(f"== {os.path.basename(os.path.dirname(path))} ({path})")
    for k, cs in sorted(agg.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        hit, miss = avg.get("TCC_HIT", 0.0), avg.get("TCC_MISS", 0.0)
        rate = hit / (hit + miss) if hit + miss else 0.0
        rd = avg.get("TCC_EA0_RDREQ", 0.0)
        print(f"{k:14s} hit={hit:.4g} miss={miss:.4g} hit_rate={rate:.3f} ea_rdreq={rd:.4g} "
              f"(x64 B = {rd * 64 / 1e9:.3f} GB) launches={len(next(iter(cs.values())))}")
