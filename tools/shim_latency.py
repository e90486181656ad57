"""Diagnostics: the drop-in shim's per-call costs on the GPU box, beside the reference's
own routing_filter.c in the same page stack (oracle/_ref/libshim_rf.so vs libref_rf.so).
Prints one JSON line (ms, median of 5):
  add_fresh_ms              routing_filter_add of 2^20 - 1 hashes
  add_incremental_ms        the same onto an existing filter (old_filter, the trunk's case)
  lookup_one_ms             one routing_filter_lookup call (per call, over 2,000 calls)
  lookup_batch_8192_ms      routing_filter_amd_lookup_batch, 8,192 (filter, key) over 8 filters
  lookup_async_8192_ms      8,192 routing_filter_lookup_async states over 8 filters, each
                            started once, then polled (the shim: one completion thread)
  async_driven_8192_ms      the same driven by callbacks, 64 in flight (test_async.c)
  async_8192_512f_ms        8,192 states over 512 filters
  mt_adds_8x_ms / 1x        8 threads each adding 2^20 - 1 hashes at once / one thread alone
                            (wall time of the adds, the keys hashed beforehand)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import refimpl as R  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402


def med(f, reps=5):
    f()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return round(float(np.median(ts)) * 1e3, 3)


out = {}
n = (1 << 20) - 1
for name, path in (("shim", R.SHIM_PATH), ("reference", R.LIB_PATH)):
    with R.Stack(path=path, cache_mib=16384, disk_mib=131072) as s:
        keys = [K.ids_keys((np.uint64(f) << np.uint64(32)) + np.arange(n, dtype=np.uint64)) for f in range(8)]
        hs = [s.hash_keys(k) for k in keys]
        base = s.add(hs[0])
        def add_phases(fn):
            """median ms of fn, and the shim's add breakdown over its runs (us per add / batch)"""
            a0 = s.add_breakdown()
            ms = med(fn)
            a1 = s.add_breakdown()
            if not a0:
                return ms, None
            d = {k: a1[k] - a0[k] for k in a0}
            c, nb = max(d["calls"], 1), max(d["batches"], 1)
            return ms, {"adds": d["calls"], "batches": d["batches"],
                        **{f"{k}_us_per_batch": round(d[f"{k}_ns"] / nb / 1e3, 1)
                           for k in ("create", "stage", "build", "infos", "readback")},
                        **{f"{k}_us_per_add": round(d[f"{k}_ns"] / c / 1e3, 1) for k in ("wait", "place")}}

        r = {}
        r["add_fresh_ms"], r["add_fresh_breakdown"] = add_phases(lambda: s.add(hs[0]))
        r["add_incremental_ms"], r["add_incremental_breakdown"] = add_phases(lambda: s.add(hs[1], value=1, old=base))
        descs = [s.add(h, value=i % 8) for i, h in enumerate(hs)]
        rng = np.random.default_rng(1)
        P = 8192
        fid = rng.integers(0, 8, size=P).astype(np.uint32)
        probe = np.stack([keys[f][rng.integers(0, n)] for f in fid])
        # one routing_filter_lookup call: 2,000 calls in a C loop (oracle/ref_harness.c
        # rfr_lookup_keys), per call -- no Python in the timed path of each call
        r["lookup_one_ms"] = round(med(lambda: s.lookup_keys(descs[0], probe[:2000]), reps=7) / 2000, 5)

        r["lookup_batch_8192_ms"] = med(lambda: s.lookup_batch(descs, probe, fid))
        st0 = s.shim_stats() or {}
        b0 = s.async_stats()
        r["lookup_async_8192_ms"] = med(lambda: s.lookup_keys_async_many(descs, probe, fid))
        st1 = s.shim_stats() or {}
        b1 = s.async_stats()
        ph = s.async_many_phases()
        r["lookup_async_8192_detail"] = {
            "start_ms": round(ph[0] / 1e6, 3), "poll_ms": round(ph[1] / 1e6, 3),
            "launches_per_call": round((b1[0] - b0[0]) / 6, 1),
            "probe_ms_per_call": round((st1.get("async_probe_ns", 0) - st0.get("async_probe_ns", 0)) / 6e6, 3)}
        ab0 = s.async_breakdown()
        r["async_driven_8192_ms"] = med(lambda: s.lookup_keys_async_driven(descs, probe, fid, max_inflight=64))
        ab1 = s.async_breakdown()
        if ab0:
            # per completion batch (6 driven runs), in microseconds
            d = {k: ab1[k] - ab0[k] for k in ab0}
            nb = max(d["batches"], 1)
            r["async_driven_breakdown"] = {
                "reaps_per_run": round(d["batches"] / 6, 1), "states_per_reap": round(d["states"] / nb, 1),
                "submit_us_per_state": round(d["submit_ns"] / max(d["states"], 1) / 1e3, 3),
                "reap_us_per_reap": round(d["reap_ns"] / nb / 1e3, 2),
                "callbacks_us_per_reap": round(d["callback_ns"] / nb / 1e3, 2),
                "run_us_per_reap": round(r["async_driven_8192_ms"] * 1e3 / max(d["batches"] / 6, 1), 2)}
        many = [s.add(s.hash_keys(K.ids_keys((np.uint64(100 + f) << np.uint64(32)) +
                                             np.arange(2000, dtype=np.uint64))), value=f % 30)
                for f in range(512)]
        fid512 = rng.integers(0, 512, size=P).astype(np.uint32)
        r["async_8192_512f_ms"] = med(lambda: s.lookup_keys_async_many(many, probe, fid512))
        T = 8
        mkeys = K.ids_keys(np.arange(T * n, dtype=np.uint64) + np.uint64(1 << 40))
        pr = K.random_keys(T * 16, seed=1)
        # the adds' wall time: the slowest thread's, hashing excluded (rfr_mt_chains)
        a0 = s.add_breakdown()
        ts8 = [float(s.mt_chains(mkeys, T, 1, n, pr, 16)[3].max()) for _ in range(3)]
        a1 = s.add_breakdown()
        if a0:
            d = {k: a1[k] - a0[k] for k in a0}
            c, nb = max(d["calls"], 1), max(d["batches"], 1)
            r["mt_adds_8x_breakdown"] = {"adds": d["calls"], "batches": d["batches"],
                                         **{f"{k}_us_per_batch": round(d[f"{k}_ns"] / nb / 1e3, 1)
                                            for k in ("create", "stage", "build", "infos", "readback")},
                                         **{f"{k}_us_per_add": round(d[f"{k}_ns"] / c / 1e3, 1)
                                            for k in ("wait", "place")}}
        ts1 = [float(s.mt_chains(mkeys[: n], 1, 1, n, pr[:16], 16)[3].max()) for _ in range(3)]
        r["mt_adds_8x_ms"] = round(float(np.median(ts8)) * 1e3, 3)
        r["mt_adds_1x_ms"] = round(float(np.median(ts1)) * 1e3, 3)
        st = s.shim_stats()
        if st:
            r["shim_stats"] = st
        out[name] = r
print(json.dumps(out), flush=True)
