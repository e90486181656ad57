"""CPU baseline for bench.py (TEST / MEASUREMENT INFRASTRUCTURE ONLY: imported by bench.py's
cpu_baseline leg alone).

What is timed:
  * the REFERENCE's own routing_filter_add / routing_filter_lookup (oracle/_ref/libref_rf.so,
    vmware/splinterdb's src/routing_filter.c and its page stack compiled unmodified, built
    with its release flags -O3 -ffast-math) -- kind "reference"; the oracle restatement
    (oracle/rf_oracle.c) only where that library is absent -- kind "port";
  * two brackets: build-only (hashes precomputed: tests/functional/filter_test.c:185-205)
    and hash + build (btree_pack's data_key_hash then routing_filter_add: what the trunk
    pays per compaction, src/btree.c:4020-4024, src/trunk.c:3821-3835), and probes;
  * one thread (one filter), and P threads = the host cores this process may use (the
    smaller of the CPU affinity set and the cgroup CPU quota), each thread building its own
    filters as SplinterDB's TASK_TYPE_NORMAL workers do (src/trunk.c:3932, :4168);
  * a calibration: the restatement timed beside the reference on the same cores, and both
    against the survey's reference timings (41 ns/key build, 53 ns/key hash +
    build, single thread, survey VM).
"""
import os

import numpy as np

SURVEY_NS_PER_KEY = {"build_only": 41.0, "hash_build": 53.0}  # SURVEY.md §6 (survey VM, 1 thread)


def host_cores():
    """(usable cores, detail): min(affinity set, cgroup v2 cpu.max quota)"""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "cpu_model": model}


def _rates(n_keys, t_hash_build, t_build_only, n_probes, t_probe):
    return {
        "hash_build_mkeys_s": round(n_keys / t_hash_build / 1e6, 2),
        "build_only_mkeys_s": round(n_keys / t_build_only / 1e6, 2),
        "probe_mkeys_s": round(n_probes / t_probe / 1e6, 2),
        "hash_build_ns_per_key": round(t_hash_build / n_keys * 1e9, 2),
        "build_only_ns_per_key": round(t_build_only / n_keys * 1e9, 2),
        "probe_ns": round(t_probe / n_probes * 1e9, 2),
    }


REPS = 2  # each bracket timed twice in a fresh reference stack; the faster run is reported


def _ref_run(lis, keys, key_len, hashes, starts, counts, threads, offs=None, probe=None):
    """reference runs: hash+build, build-only, probes (best of REPS, each in a fresh stack).
    probe = (keys, offs, filter ids) or None for the build keys themselves (each probing its
    own filter)."""
    from oracle import refimpl as R
    best = None
    for _ in range(REPS):
        with R.Stack(log_index_size=lis, cache_mib=4096, disk_mib=65536) as s:
            t_hb, keep = s.bench_build(keys, key_len, starts, counts, threads, hash_keys=True, offs=offs)
            if probe is None:
                fid = np.repeat(np.arange(len(counts), dtype=np.uint32), counts)
                t_pr, found = s.bench_probe(keep, keys, key_len, fid, threads, offs=offs)
            else:
                t_pr, found = s.bench_probe(keep, probe[0], key_len, probe[2], threads, offs=probe[1])
            assert s.device_writes() == 0
        with R.Stack(log_index_size=lis, cache_mib=4096, disk_mib=65536) as s:
            t_bo, _ = s.bench_build(hashes, 4, starts, counts, threads, hash_keys=False)
        r = (t_hb, t_bo, t_pr, found)
        best = r if best is None else tuple(min(a, b) for a, b in zip(best[:3], r[:3])) + (found,)
    return best


def _port_run(lis, keys, key_len, hashes, starts, counts, threads):
    best = None
    for _ in range(REPS):
        r = _port_once(lis, keys, key_len, hashes, starts, counts, threads)
        best = r if best is None else tuple(min(a, b) for a, b in zip(best[:3], r[:3])) + (r[3],)
    return best


def _port_once(lis, keys, key_len, hashes, starts, counts, threads):
    import ctypes
    from oracle import oracle as O
    ocfg = O.make_config(log_index_size=lis)
    L = O.lib()
    nf = len(counts)
    st = np.ascontiguousarray(starts, dtype=np.uint64)
    ct = np.ascontiguousarray(counts, dtype=np.uint32)
    keep = (O.Filter * nf)()
    t_hb = L.rfo_bench_build(ctypes.byref(ocfg), keys.ctypes.data, key_len, 1, st.ctypes.data, ct.ctypes.data,
                             nf, 0, threads, keep)
    keep2 = (O.Filter * nf)()
    t_bo = L.rfo_bench_build(ctypes.byref(ocfg), hashes.ctypes.data, 4, 0, st.ctypes.data, ct.ctypes.data,
                             nf, 0, threads, keep2)
    fid = np.repeat(np.arange(nf, dtype=np.uint32), counts)
    found = np.zeros(fid.size, dtype=np.uint64)
    t_pr = L.rfo_bench_probe(ctypes.byref(ocfg), keep, keys.ctypes.data, key_len, fid.ctypes.data, fid.size,
                             threads, found.ctypes.data)
    for i in range(nf):
        L.rfo_filter_release(ctypes.byref(keep[i]))
        L.rfo_filter_release(ctypes.byref(keep2[i]))
    return t_hb, t_bo, t_pr, found


def fixed_keys(lis, n, threads=0):
    """C2-C4: filters of n sequential-id 24 B keys (filter_test format). Single thread: one
    filter; all cores: one filter per thread."""
    from oracle import oracle as O
    from oracle import refimpl as R
    from splinterdb_amd import keys as K
    cores, host = host_cores()
    P = threads or cores
    keys = K.seq_keys(0, P * n)
    hashes = O.hash_fixed(keys.reshape(-1), 24)
    starts = np.arange(P, dtype=np.uint64) * n
    counts = np.full(P, n, dtype=np.uint32)
    kind = "reference" if R.available() else "port"
    run = _ref_run if kind == "reference" else _port_run
    one = run(lis, keys[:n], 24, hashes[:n], starts[:1], counts[:1], 1)
    allc = run(lis, keys, 24, hashes, starts, counts, P)
    ok = bool((allc[3] & np.uint64(1)).all()) and bool((one[3] & np.uint64(1)).all())
    single = _rates(n, one[0], one[1], n, one[2])
    multi = _rates(P * n, allc[0], allc[1], P * n, allc[2])
    out = {
        "value": round(P * n / (allc[0] + allc[2]) / 1e6, 2),
        "unit": "Mkeys/s",
        "cores": P,
        "kind": kind,
        "sample": f"{P} filters x {n} keys (24 B seq ids), one filter per thread on {P} threads: "
                  f"hash + routing_filter_add ({allc[0]:.2f} s), then routing_filter_lookup of all "
                  f"{P * n} keys ({allc[2]:.2f} s); build-only and 1-thread brackets below; "
                  f"no false negatives: {ok}",
        "host": host,
        "all_cores": dict(threads=P, filters=P, keys_per_filter=n, **multi),
        "single_thread": dict(filters=1, keys_per_filter=n, **single),
        "build_mkeys_s": multi["hash_build_mkeys_s"],
        "probe_mkeys_s": multi["probe_mkeys_s"],
    }
    cal = {"survey_reference_ns_per_key_1thread": SURVEY_NS_PER_KEY}
    if kind == "reference":
        port = _port_run(lis, keys[:n], 24, hashes[:n], starts[:1], counts[:1], 1)
        ps = _rates(n, port[0], port[1], n, port[2])
        cal["port_single_thread"] = ps
        cal["port_over_reference_ns"] = {
            "hash_build": round(ps["hash_build_ns_per_key"] / single["hash_build_ns_per_key"], 3),
            "build_only": round(ps["build_only_ns_per_key"] / single["build_only_ns_per_key"], 3),
            "probe": round(ps["probe_ns"] / single["probe_ns"], 3)}
    cal["reference_here_over_survey_ns"] = {
        "hash_build": round(single["hash_build_ns_per_key"] / SURVEY_NS_PER_KEY["hash_build"], 3),
        "build_only": round(single["build_only_ns_per_key"] / SURVEY_NS_PER_KEY["build_only"], 3)}
    out["calibration"] = cal
    return out


def var_keys(lis, w, F, n, threads=0):
    """C5: the whole variable-length workload: F filters of n keys, and its probe mix"""
    from oracle import refimpl as R
    cores, host = host_cores()
    P = threads or cores
    starts = np.arange(F, dtype=np.uint64) * n
    counts = np.full(F, n, dtype=np.uint32)
    if not R.available():
        return None
    with R.Stack(log_index_size=lis) as s:
        hashes = s.hash_var_keys(w["bytes"], w["offs"])
    Pp = w["probe_fid"].size
    t_hb, t_bo, t_pr, found = _ref_run(lis, w["bytes"], 0, hashes, starts, counts, P, offs=w["offs"],
                                       probe=(w["probe_bytes"], w["probe_offs"], w["probe_fid"]))
    ok = bool((found[w["positive"]] & np.uint64(1)).all())
    total = F * n
    rates = _rates(total, t_hb, t_bo, Pp, t_pr)
    return {
        "value": round(total / (t_hb + t_pr) / 1e6, 2), "unit": "Mkeys/s", "cores": P, "kind": "reference",
        "sample": f"the whole C5 workload: {F} filters x {n} variable-length keys, hash + routing_filter_add "
                  f"one filter per thread on {P} threads ({t_hb:.2f} s), routing_filter_lookup of {Pp} mixed "
                  f"probes ({t_pr:.2f} s); positives found: {ok}",
        "host": host, "all_cores": dict(threads=P, filters=F, keys_per_filter=n, **rates),
        "build_mkeys_s": rates["hash_build_mkeys_s"], "probe_mkeys_s": rates["probe_mkeys_s"],
    }


def chain(lis, rounds, n, threads=0):
    """bench.py --workload compaction: the reference's own incremental routing_filter_add
    chains (oracle/ref_harness.c chain_worker: keys generated and hashed per round, old filter
    merged, superseded filter dec_ref'd), one chain per thread on every usable core, and one
    chain on one thread."""
    from oracle import refimpl as R
    if not R.available():
        return None
    cores, host = host_cores()
    P = threads or cores
    best = {}
    for label, nf, th in (("all_cores", P, P), ("single_thread", 1, 1)):
        t_best = None
        for _ in range(REPS):
            with R.Stack(log_index_size=lis, cache_mib=8192, disk_mib=131072) as s:
                t, keep = s.bench_chain(nf, rounds, n, th)
                u0 = int(keep[0].num_unique)
                for f in range(nf):
                    s.dec_ref(keep[f])
            t_best = t if t_best is None else min(t_best, t)
        best[label] = {"threads": th, "chains": nf, "seconds": round(t_best, 3),
                       "mkeys_s": round(nf * rounds * n / t_best / 1e6, 2),
                       "ns_per_key": round(t_best / (nf * rounds * n) * 1e9 * th, 1)}
    return {
        "value": best["all_cores"]["mkeys_s"], "unit": "Mkeys/s", "cores": P, "kind": "reference",
        "sample": f"{P} chains (one per thread on {P} threads) of {rounds} incremental routing_filter_adds of "
                  f"{n} 24 B keys each (keys generated + hashed per round, superseded filter dec_ref'd); "
                  f"filter 0's num_unique {u0}",
        "host": host, "all_cores": best["all_cores"], "single_thread": best["single_thread"],
    }
