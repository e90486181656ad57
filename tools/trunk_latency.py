"""Diagnostics: the reference's own key-value store (oracle/ref_kvs.c) with its
routing_filter.c and with the drop-in shim, same workload: insert wall time (the trunk's
filter builds included), per-lookup latency of splinterdb_lookup and of core_lookup_async at
64 in flight, filter calls per lookup; stores driven as the unmodified reference drives them and with the
shim's cache attach. One JSON line.
usage: python tools/trunk_latency.py [n_keys] [memtable_mib]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import refkvs as RK  # noqa: E402
from test_ref_kvs import workload  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
mt = int(sys.argv[2]) if len(sys.argv) > 2 else 8
keys, vals, absent = workload(n, seed=11)
rng = np.random.default_rng(5)
P = 50_000
probe_hit = keys[rng.choice(n, P, replace=False)]
probe_miss = absent[:P]
out = {"keys": n, "memtable_mib": mt, "probes": P}
for name, path in (("reference", RK.KVS_REF), ("shim", RK.KVS_SHIM)):
    # three stores one after another in this process: "first" and "second" are driven as the
    # unmodified reference drives the filter (no shim extension called: the bounce-buffer path;
    # the first store of the process also pays the shim's engine creation inside its first
    # routing_filter_add), "attached" calls routing_filter_amd_cache_attach after opening (its
    # page buffer registered: images placed straight into the cache pages) and release before
    # closing. Lookups are timed on the second store.
    out[name] = {}
    for run, attach in (("first", False), ("second", False), ("attached", True)):
        with RK.Kvs(path, memtable_mib=mt, record_digest=False, attach=attach) as db:
            b0 = db.add_breakdown()
            t = time.perf_counter()
            db.insert(keys, vals)
            ins = time.perf_counter() - t
            b1 = db.add_breakdown()
            recs, nl0, na0 = db.adds()
            bd = {k: round((b1[k] - b0[k]) / 1e6, 3) for k in b1 if k not in ("calls", "batches")}
            ds = db.direct_stats()
            r = {"insert_s": round(ins, 3), "filter_adds": int(len(recs)), "add_breakdown_ms": bd,
                 "direct_stats": [int(x) for x in ds[:3]]}
            if attach:
                r["attached"] = db.attached
                r["attach_s"] = round(db.attach_s, 3)
            if run == "second":
                r["filter_fps_added"] = int(recs["num_new"].sum()) if len(recs) else 0
                for kind, pr in (("hit", probe_hit), ("miss", probe_miss)):
                    f, _, ts = db.lookup(pr)
                    _, nl1, _ = db.adds()
                    fa, _, ta = db.lookup_async(pr, 64)
                    _, nl2, na2 = db.adds()
                    r[f"lookup_{kind}_us"] = round(ts / P * 1e6, 3)
                    r[f"lookup_async64_{kind}_us"] = round(ta / P * 1e6, 3)
                    r[f"filter_lookups_per_{kind}"] = round((nl1 - nl0) / P, 2)
                    r[f"found_{kind}"] = int(f.sum())
                    nl0 = nl2
            out[name][run] = r
print(json.dumps(out))
