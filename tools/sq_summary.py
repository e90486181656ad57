"""Per-kernel SQ counter summary from a rocprofv3 --pmc counter_collection.csv (diagnostics).
Prints per-launch averages and, for VALU/LDS, the implied SIMD cycles per CU.
usage: python tools/sq_summary.py <counter_collection.csv> [num_CUs=256]"""
import collections
import csv
import sys

sys.path.insert(0, "profiles")
from pmc_summary import short  # noqa: E402

path = sys.argv[1]
cus = int(sys.argv[2]) if len(sys.argv) > 2 else 256
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(path)):
    s = short(r["Kernel_Name"]) or r["Kernel_Name"].split("(")[0][:24]
    agg[s][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    line = " ".join(f"{c.replace('SQ_', '')}={v:.3g}" for c, v in sorted(avg.items()))
    extra = ""
    if "SQ_INSTS_VALU" in avg:
        # a wave64 VALU instruction occupies a SIMD for >= 4 cycles (16 lanes wide)
        extra += f" | VALU cyc/SIMD >= {avg['SQ_INSTS_VALU'] * 4 / (4 * cus):.0f}"
    if "SQ_INSTS_LDS" in avg:
        extra += f" | LDS instr/CU {avg['SQ_INSTS_LDS'] / cus:.0f}"
    print(f"{k:14s} {line}{extra}")
