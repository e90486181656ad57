"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE collected in separate runs, as
MI355X_MICROARCH.md prescribes) into per-launch HBM bytes per kernel.

Corrections (MI355X_MICROARCH.md §HBM): rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB;
on gfx950 FETCH_SIZE reads exactly 1/2 of the bytes of a wide coalesced streaming read, so
the fetch side is doubled ("fetch_x2"); WRITE_SIZE is exact for 16-B-per-lane streaming
stores. Kernels whose reads are random 16-B windows (k_probe) are NOT calibrated by that
rule -- both the raw and the doubled figure are kept, and bench.py uses the raw + write
figure as a lower bound for them.

usage: python profiles/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
"""
import collections
import csv
import json
import sys

SHORT = {"k_hash_scatter": "partition", "k_hash_count": "count_fallback", "k_scatter": "scatter_fallback",
         "k_cb_sort<": "cb_sort", "k_cb_sort_big": "cb_sort_big", "k_layout": "layout",
         "k_assemble": "assemble", "k_plines": "plines", "k_probe": "probe", "k_cb_scan": "count_scan"}


def short(name):
    for k, v in SHORT.items():
        if k in name.split("(")[0]:
            return v
    return None


def load(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        s = short(r["Kernel_Name"])
        if s:
            agg[s].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in agg.items()}


if __name__ == "__main__":
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    out = {"source": sys.argv[1:3], "unit": "bytes per launch",
           "fetch_raw": f, "fetch_x2": {k: 2 * v for k, v in f.items()}, "write": w,
           "per_launch_hbm_bytes": {}}
    for k in f:
        streaming = k != "probe"
        out["per_launch_hbm_bytes"][k] = int((2 * f[k] if streaming else f[k]) + w.get(k, 0))
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, v in sorted(out["per_launch_hbm_bytes"].items()):
        print(f"{k:12s} fetch_raw {f[k]/1e6:9.1f} MB  write {w.get(k,0)/1e6:9.1f} MB  hbm {v/1e6:9.1f} MB")
