#!/usr/bin/env python3
"""Routing-filter benchmark (BASELINE.json metric: routing_filter build Mkeys/s + probe
Mkeys/s, device-resident, 24 B keys).

Workload = BASELINE config 2 per GPU: 64M x 24 B keys as 8 filters x 8,000,000 keys (the
per-filter cap at log_index_size 8 is 8,388,607, src/routing_filter.h:120-127), fp_size
26, seed 42, sequential-id keys in the reference's filter_test format. One STEP = build all
8 filters from the device-resident keys (hash -> bucket -> encode -> pack pages) AND probe
all 64M keys against their filters. value = keys / step time (both phases), whole job.

Multi-GPU: one process per GPU (torchrun); each rank owns a contiguous key range and its
own 8 filters (SplinterDB filters are per key-range, src/trunk.c:4133-4170), so there is
no data-path collective: scaling is weak, time = max over ranks, value = all ranks' keys
/ that time.

CPU baseline (rank 0, N=1; oracle/cpu_baseline.py): the reference's own routing_filter_add /
routing_filter_lookup (oracle/_ref/libref_rf.so: src/routing_filter.c and its page stack
compiled unmodified) on a bounded sample of the same workload -- one filter per thread on
every usable host core like SplinterDB's background tasks, and on one thread -- in
build-only and hash + build brackets, with the oracle restatement timed beside it as a
calibration.

`--gpus N` (N > 1) without torchrun starts the N ranks itself (launch_ranks).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from splinterdb_amd import engine as E  # noqa: E402
from splinterdb_amd import keys as K  # noqa: E402
from splinterdb_amd import route as R  # noqa: E402
from splinterdb_amd import shard as S  # noqa: E402

WORKLOADS = {
    # name: (filters, keys per filter, scaling, description)
    "c2": (8, 8_000_000, "weak", "C2: 64M x 24B keys per GPU = 8 filters x 8,000,000, build + full probe"),
    "c3": (256, 1 << 20, "weak", "C3: 256M x 24B keys per GPU = 256 filters x 2^20, build + full probe"),
    "c4": (1024, 1 << 20, "strong", "C4: 2^30 x 24B keys = 1024 filters x 2^20 split by key range, build + full probe"),
    "c5": (8, 1 << 21, "weak", "C5: 16.8M variable-length (8-100 B) keys per GPU = 8 filters x 2^21, build + "
                               "as many probes (90% Zipf(0.99) positives, 10% negatives, shuffled)"),
    "compaction": (64, (1 << 20) - 1, "weak",
                   "compaction chains: 64 filters per GPU, each grown by 8 incremental routing_filter_adds of "
                   "2^20-1 keys (filter_test's basic chain, keys (f << 32) + (v + 1) j, value v); every round = "
                   "create + build (merging the previous round's filter) + release of the superseded filter; "
                   "images device-resident (a PCIe-inclusive chain with every round's pages read back is "
                   "reported beside)"),
}
CHAIN_ROUNDS = 8

METRIC = "routing_filter build Mkeys/s + probe Mkeys/s, device-resident, 24B keys"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=list(WORKLOADS), default="c2",
                   help="c2: 8 x 8,000,000 keys per GPU (weak); c3: 256 x 2^20 per GPU (weak); "
                        "c4: 1024 x 2^20 keys in total, split over the GPUs (strong); "
                        "c5: 8 x 2^21 variable-length keys per GPU + Zipf probe mix (weak); "
                        "compaction: 64 incremental chains of 8 x (2^20-1) keys per GPU (weak; "
                        "a step = one whole chain)")
    p.add_argument("--filters", type=int, default=0, help="override filters (per GPU for c2/c3)")
    p.add_argument("--keys-per-filter", type=int, default=0)
    p.add_argument("--log-index-size", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU baseline threads (0 = every usable core: the affinity set capped by the cgroup quota)")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--dist-always", action="store_true",
                   help="initialise torch.distributed (RCCL) and run every collective even with one rank: "
                        "exercises the multi-rank code path on a one-GPU box")
    p.add_argument("--routed-probe", action="store_true",
                   help="also time routed probes: each rank probes keys of every rank's filters, "
                        "moved to the owner by all-to-all (route.py); reported beside value")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_r05.json"))
    p.add_argument("--digest-out", default="",
                   help="write each rank's per-filter image SHA-256s to <path>.rank<r> (tests)")
    return p.parse_args()


def stage_bytes(stage, N, P, image_bytes, slot_bytes, unique, key_bytes=None, probe_key_bytes=None):
    """Algorithmic bytes per launch of each stage (DESIGN.md 'Roofline'). Fixed 24 B keys
    unless key_bytes / probe_key_bytes give the variable-length totals (bytes + offsets)."""
    kb = N * 24 if key_bytes is None else key_bytes
    pkb = P * 24 if probe_key_bytes is None else probe_key_bytes
    return {
        "partition": kb + N * 4,               # fused K1+K3: read keys, write bucketed entries
        "cb_sort": N * 4 + unique * 4,         # read bucketed entries, write sorted unique
        "assemble": unique * 4 + image_bytes,  # read sorted entries, write pages
        "probe": pkb + P * 8 + image_bytes + slot_bytes,  # SURVEY.md §8(d) probe figure
    }.get(stage)


def cpu_baseline(args, cfg_lis, n):
    """The reference's own routing_filter_add / routing_filter_lookup on this host's cores
    (oracle/cpu_baseline.py): single thread and all usable cores, build-only and hash +
    build brackets, probes, and the restatement's calibration against the reference."""
    from oracle import cpu_baseline as CB
    return CB.fixed_keys(cfg_lis, n, threads=args.cpu_threads)


def cpu_baseline_var(args, cfg_lis, w, F, n):
    """C5: the reference over the whole variable-length workload and its probe mix."""
    from oracle import cpu_baseline as CB
    return CB.var_keys(cfg_lis, w, F, n, threads=args.cpu_threads)


def launch_ranks(args):
    """`--gpus N` is the number of ranks, one per GPU. Under torchrun (WORLD_SIZE set) it
    must agree with WORLD_SIZE. Without it, N > 1 starts the N ranks here: a child
    torch.distributed.run on 127.0.0.1, started before this process makes any HIP call (no
    exec from a process that touched the GPU). Returns the children's exit status, or None
    when this process is itself the (only) rank."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
        return None
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if args.gpus == 1:
        return None
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def e2e_duplex(eng, cfg, stream, ins, h_ins, compute, found, batch, infos, n, F, N, P, found_ok, reps=6):
    """PCIe-inclusive rate of a stream of `reps` batches with two in flight (full duplex):
    inputs H2D on a copy-in stream, build + probe on `stream`, found_values + page images +
    index slots D2H on a copy-out stream, every buffer double-buffered. `ins` are the device
    input tensors (keys; or C5's key bytes, offsets, probe bytes, offsets and filter ids),
    `h_ins` their pinned host sources, compute(batch, ins, found) issues one build + probe on
    `stream`, found_ok(host found) checks the results. Returns (Mkeys/s of this rank, the
    results checked and both batches' images equal)."""
    dev = found.device
    s_in, s_out = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    ib = [list(ins), [torch.empty_like(x) for x in ins]]
    fb = [found, torch.empty_like(found)]
    batch2 = E.FilterBatch(cfg, [n] * F, engine=eng)
    bb = [batch, batch2]
    hf = [torch.empty(P, dtype=torch.int64).pin_memory() for _ in range(2)]
    hp = [[torch.empty(i.num_pages * cfg.page_size, dtype=torch.uint8).pin_memory() for i in infos] for _ in range(2)]
    hs = [[torch.empty(i.num_indices, dtype=torch.int64).pin_memory() for i in infos] for _ in range(2)]
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_comp = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]

    def one(r):
        s = r % 2
        if r >= 2:
            s_in.wait_event(ev_comp[s])  # batch r-2 read these inputs
        with torch.cuda.stream(s_in):
            for d, h in zip(ib[s], h_ins):
                d.view(-1).copy_(h.view(-1), non_blocking=True)
        ev_in[s].record(s_in)
        stream.wait_event(ev_in[s])
        if r >= 2:
            stream.wait_event(ev_out[s])  # batch r-2's results and images have left
        compute(bb[s], ib[s], fb[s])
        ev_comp[s].record(stream)
        s_out.wait_event(ev_comp[s])
        with torch.cuda.stream(s_out):
            hf[s].copy_(fb[s], non_blocking=True)
        for f in range(F):
            bb[s].read_image_async(f, hp[s][f], hs[s][f], s_out.cuda_stream)
        ev_out[s].record(s_out)

    one(0)  # warm-up (the second batch's first build)
    one(1)
    torch.cuda.synchronize()
    te = time.perf_counter()
    for r in range(reps):
        one(r)
    torch.cuda.synchronize()
    rate = N * reps / (time.perf_counter() - te) / 1e6
    ok = all(found_ok(hf[s]) for s in range(2))
    # both batches' images equal (the same keys)
    ok = ok and all(torch.equal(hp[0][f], hp[1][f]) and torch.equal(hs[0][f], hs[1][f]) for f in range(F))
    batch2.close()
    return rate, ok


def main():
    args = parse()
    spawned = launch_ranks(args)
    if spawned is not None:
        sys.exit(spawned)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU; RF_BENCH_BACKEND=gloo (and ranks sharing a device) only to rehearse
    # the multi-rank launch on a one-GPU box -- the data path has no collective either way
    backend = os.environ.get("RF_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % max(1, ndev)
    if world > 1 or args.dist_always:
        import torch.distributed as dist
        if world == 1 and "MASTER_PORT" not in os.environ:  # one rank without torchrun
            import socket
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll_dev = dev if backend == "nccl" else None  # device of the timing reductions

    if args.workload == "compaction":
        return run_compaction(args, rank, world, dist, dev, coll_dev, backend)

    wf, wn, scaling, wdesc = WORKLOADS[args.workload]
    var = args.workload == "c5"
    n = args.keys_per_filter or wn
    if scaling == "weak":
        F_total = (args.filters or wf) * world
    else:
        F_total = args.filters or wf
    me = S.plan_shards(F_total, n, world)[rank]
    F = me.num_filters
    N = me.num_keys
    cfg = E.routing_config_init(fingerprint_size=26, log_index_size=args.log_index_size, seed=42)
    eng = E.Engine(local)
    stream = torch.cuda.Stream(device=dev)
    w = None
    key_bytes = probe_key_bytes = None
    with torch.cuda.stream(stream):
        if var:
            # C5: host-generated variable-length keys + Zipf probe mix, copied to HBM once
            w = K.c5_inputs(F, n, seed=0x5EED + me.key_begin)
            d_bytes, d_offs = torch.from_numpy(w["bytes"]).to(dev), torch.from_numpy(w["offs"].view(np.int64)).to(dev)
            p_bytes = torch.from_numpy(w["probe_bytes"]).to(dev)
            p_offs = torch.from_numpy(w["probe_offs"].view(np.int64)).to(dev)
            fid = torch.from_numpy(w["probe_fid"].view(np.int32)).to(dev)
            positive = torch.from_numpy(w["positive"]).to(dev)
            P = int(w["probe_fid"].size)
            key_bytes = w["bytes"].nbytes + w["offs"].nbytes
            probe_key_bytes = w["probe_bytes"].nbytes + w["probe_offs"].nbytes + 4 * P
        else:
            # key-range shard of this rank: ids [key_begin, key_end), filter f = ids of its range
            keys = K.seq_keys_torch(me.key_begin, N, 24, dev)
            counts = [n] * F  # probes grouped by filter: filter f's keys probe filter f
            P = N
        found = torch.empty(P, dtype=torch.int64, device=dev)
    stream.synchronize()
    batch = E.FilterBatch(cfg, [n] * F, engine=eng)
    # one event set per timed step, read after the timed loop (the loop never waits on the
    # host). The timed steps record only the probe's two events (the roofline's kernel time):
    # an event between every build kernel costs the C2 step ~40 us (tools/event_cost.py), so
    # the per-kernel build times come from a separate pass after the timed loop.
    batch.set_timing(True, sets=max(1, args.steps), probe_only=True)

    def step():
        if var:
            batch.build_var_keys(d_bytes, d_offs, stream=stream.cuda_stream)
            batch.probe_var_keys(p_bytes, p_offs, fid, P, found, stream=stream.cuda_stream)
        else:
            batch.build_keys(keys, 24, stream=stream.cuda_stream)
            batch.probe_keys_runs(keys, 24, counts, found, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    stream.synchronize()
    stages = {k: [] for k in E.FilterBatch.STAGES}

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    for back in range(args.steps):  # the probe's HIP events of every timed step, on its stream
        stages["probe"].append(batch.timings(back)["probe"])
    # per-kernel build stages: a short pass with an event between every kernel (not timed)
    diag = min(args.steps, 5)
    batch.set_timing(True, sets=diag)
    for _ in range(diag):
        step()
    stream.synchronize()
    for back in range(diag):
        for k, v in batch.timings(back).items():
            if k != "probe":
                stages[k].append(v)
    elapsed = S.max_over_ranks(elapsed, dist, coll_dev)
    keys_all = S.sum_over_ranks(float(N), dist, coll_dev)

    # ---- verification (outside the timed region) -------------------------------------
    if var:
        ok = bool(((found[positive] & 1) == 1).all().item())
    else:
        ok = bool(((found & 1) == 1).all().item())
    # ---- the probe's measured memory floor (after the results were checked: it overwrites
    # `found`): the fast path's key staging, line gather and store over the same runs with the
    # hash and decode removed (rf_amd_debug_probe_floor), HIP events on the probe's stream
    floor_ms = None
    if not var:
        batch.probe_floor(keys, 24, counts, found, stream=stream.cuda_stream)
        fe = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        freps = 5
        fe[0].record(stream)
        for _ in range(freps):
            batch.probe_floor(keys, 24, counts, found, stream=stream.cuda_stream)
        fe[1].record(stream)
        stream.synchronize()
        floor_ms = S.max_over_ranks(fe[0].elapsed_time(fe[1]) / freps, dist, coll_dev)
    infos = [batch.info(f) for f in range(F)]
    image_bytes = sum(i.num_pages for i in infos) * cfg.page_size
    slot_bytes = sum(i.num_indices for i in infos) * 8
    unique = sum(i.num_unique for i in infos)
    verified = ok and all(i.error == 0 for i in infos)
    # image bytes against the committed golden SHA-256s (tests/golden/sha256.json, made by
    # oracle/gen_golden.py) for every filter of this rank that has one: C2's filter 0, and
    # the sampled C3/C4 filters k of the 2^20-key layout (ids [k 2^20, (k+1) 2^20))
    sha_checked = []
    if not var and args.log_index_size == 8:
        with open(os.path.join(ROOT, "tests", "golden", "sha256.json")) as fh:
            gold = json.load(fh)
        for f in range(F):
            g = me.filter_begin + f
            key = ("seq_n8000000_lis8" if n == 8_000_000 and g == 0 else
                   f"seq_n{n}_lis8_k{g}" if n == 1 << 20 else None)
            if key in gold:
                img = batch.image(f)
                good = (hashlib.sha256(img.pages.tobytes()).hexdigest() == gold[key]["pages_sha256"] and
                        hashlib.sha256(img.slots.tobytes()).hexdigest() == gold[key]["slots_sha256"])
                verified = verified and good
                sha_checked.append(g)
    if args.digest_out:
        # per-filter image digests of this rank (the multi-rank tests compare them with a
        # single-process build of the same filters)
        dig = {}
        for f in range(F):
            img = batch.image(f)
            dig[me.filter_begin + f] = hashlib.sha256(img.pages.tobytes() + img.slots.tobytes()).hexdigest()
        with open(f"{args.digest_out}.rank{rank}", "w") as fh:
            json.dump(dig, fh)

    # ---- end-to-end (PCIe-inclusive) rate, reported beside `value` (never as it) ------
    # keys H2D from pinned host memory -> build -> probe -> found_values + page images +
    # index slots D2H into pinned host buffers (the clockcache page buffers' stand-in).
    e2e = e2e_h = e2e_serial = None
    if not args.no_e2e:
        if var:
            h_in = [(d_bytes, torch.from_numpy(w["bytes"]).pin_memory()),
                    (d_offs, torch.from_numpy(w["offs"].view(np.int64)).pin_memory()),
                    (p_bytes, torch.from_numpy(w["probe_bytes"]).pin_memory()),
                    (p_offs, torch.from_numpy(w["probe_offs"].view(np.int64)).pin_memory()),
                    (fid, torch.from_numpy(w["probe_fid"].view(np.int32)).pin_memory())]
        else:
            h_in = [(keys.view(-1), torch.from_numpy(K.seq_keys(me.key_begin, N).reshape(-1)).pin_memory())]
        hfound = torch.empty(P, dtype=torch.int64).pin_memory()
        hpages = [torch.empty(i.num_pages * cfg.page_size, dtype=torch.uint8).pin_memory() for i in infos]
        hslots = [torch.empty(i.num_indices, dtype=torch.int64).pin_memory() for i in infos]
        reps = 3
        torch.cuda.synchronize()
        te = time.perf_counter()
        for _ in range(reps):
            with torch.cuda.stream(stream):
                for d, h in h_in:
                    d.copy_(h, non_blocking=True)
            step()
            with torch.cuda.stream(stream):
                hfound.copy_(found, non_blocking=True)
            for f in range(F):
                batch.read_image_async(f, hpages[f], hslots[f], stream.cuda_stream)
        stream.synchronize()
        e2e_serial = S.sum_over_ranks(N * reps / (time.perf_counter() - te) / 1e6, dist, coll_dev)
        if var:
            ok_e2e = bool(((hfound[torch.from_numpy(w["positive"])] & 1) == 1).all().item())
        else:
            ok_e2e = bool(((hfound & 1) == 1).all().item())
        verified = verified and ok_e2e
        e2e = e2e_serial
        # full duplex: a stream of batches, two in flight -- batch r+1's keys cross PCIe
        # host->device (copy-in stream) while batch r's results and images cross
        # device->host (copy-out stream) and the GPU builds and probes in between; inputs,
        # results, images and the filter batch are double-buffered
        if var:
            pos = torch.from_numpy(w["positive"])

            def compute(b, ins, fo):
                b.build_var_keys(ins[0], ins[1], stream=stream.cuda_stream)
                b.probe_var_keys(ins[2], ins[3], ins[4], P, fo, stream=stream.cuda_stream)

            def found_ok(hf):
                return bool(((hf[pos] & 1) == 1).all().item())
        else:
            def compute(b, ins, fo):
                b.build_keys(ins[0], 24, stream=stream.cuda_stream)
                b.probe_keys_runs(ins[0], 24, counts, fo, stream=stream.cuda_stream)

            def found_ok(hf):
                return bool(((hf & 1) == 1).all().item())
        e2e, ok_dup = e2e_duplex(eng, cfg, stream, [d for d, _ in h_in], [h for _, h in h_in], compute, found,
                                 batch, infos, n, F, N, P, found_ok)
        e2e = S.sum_over_ranks(e2e, dist, coll_dev)
        verified = verified and ok_dup
        if not var:
            # the drop-in interface itself takes fingerprints, not keys (routing_filter_add's
            # new_fp_arr; btree_pack hashes on the host): 4 B/key H2D instead of 24
            with torch.cuda.stream(stream):
                d_h = torch.empty(N, dtype=torch.int32, device=dev)
            E.hash_keys(cfg, keys, 24, N, d_h, stream=stream.cuda_stream, engine=eng)
            stream.synchronize()
            hh = d_h.cpu().pin_memory()
            torch.cuda.synchronize()
            te = time.perf_counter()
            for _ in range(reps):
                with torch.cuda.stream(stream):
                    d_h.copy_(hh, non_blocking=True)
                batch.build_hashes(d_h, stream=stream.cuda_stream)
                batch.probe_hashes_runs(d_h, counts, found, stream=stream.cuda_stream)
                with torch.cuda.stream(stream):
                    hfound.copy_(found, non_blocking=True)
                for f in range(F):
                    batch.read_image_async(f, hpages[f], hslots[f], stream.cuda_stream)
            stream.synchronize()
            e2e_h = S.sum_over_ranks(N * reps / (time.perf_counter() - te) / 1e6, dist, coll_dev)
            verified = verified and bool(((hfound & 1) == 1).all().item())

    # ---- routed probes (serving across ranks, reported beside `value`, never as it) ------
    # probe i of rank r looks up global key id (i * world + r) mod total: every rank's probes
    # cover every rank's filters, so (world-1)/world of them cross to another GPU and back
    routed = None
    if args.routed_probe and not var:
        total_keys = F_total * n
        gid = (torch.arange(N, device=dev, dtype=torch.int64) * world + rank) % total_keys
        rkeys = K.ids_keys_torch(gid, 24)
        rfid = (gid // n).to(torch.int32)
        del gid
        d_rh = torch.empty(N, dtype=torch.int32, device=dev)
        rfound = torch.zeros(N, dtype=torch.int64, device=dev)
        router = R.ProbeRouter(S.plan_shards(F_total, n, world), rank, batch, dev, dist=dist,
                               coll_device=coll_dev if coll_dev is not None else "cpu",
                               ops=R.GpuRouteOps(eng), collective_at_one=args.dist_always)
        reps = max(1, min(args.steps, 5))

        def rstep():
            with torch.cuda.stream(stream):
                E.hash_keys(cfg, rkeys, 24, N, d_rh, stream=stream.cuda_stream, engine=eng)
                router.lookup_hashes(d_rh, rfid, N, rfound)

        rstep()
        stream.synchronize()
        barrier()
        tr = time.perf_counter()
        for _ in range(reps):
            rstep()
        stream.synchronize()
        barrier()
        tr = S.max_over_ranks(time.perf_counter() - tr, dist, coll_dev)
        r_ok = bool(((rfound & 1) == 1).all().item())
        r_ok = S.max_over_ranks(0.0 if r_ok else 1.0, dist, coll_dev) == 0.0  # every rank's probes
        routed = {"mkeys_s": round(keys_all * reps / tr / 1e6, 1), "ms": round(tr / reps * 1e3, 3),
                  "reps": reps, "verified": r_ok,
                  "exchange": "none (1 rank)" if (world == 1 and not args.dist_always) else
                  ("all-to-all over RCCL" if coll_dev is not None else "all-to-all over gloo (rehearsal)")
                  + (" (1 rank)" if world == 1 else "")}
        del rkeys, rfid, d_rh, rfound, router

    # every rank's checks, not only rank 0's: the line says verified only if all ranks agree
    verified = S.max_over_ranks(0.0 if verified else 1.0, dist, coll_dev) == 0.0
    ms = {k: float(np.mean(v)) for k, v in stages.items()}
    kern = {}
    for k in ("partition", "count_scan", "scatter", "cb_sort", "cb_sort_big", "layout", "assemble", "probe"):
        b = stage_bytes(k, N, P, image_bytes, slot_bytes, unique, key_bytes, probe_key_bytes)
        kern[k] = {"ms": round(ms[k], 4), "events": "timed steps" if k == "probe" else "stage pass"}
        if b:
            kern[k]["alg_bytes"] = int(b)
            kern[k]["gbs"] = round(b / (ms[k] * 1e-3) / 1e9, 1) if ms[k] > 0 else None
    # the dominant kernel, the same on every rank (the slowest rank's times decide), and its
    # roofline for the whole job: every rank's algorithmic bytes over the slowest rank's
    # kernel time, against world x one GPU's peak (fraction of G x roofline)
    cand = ("partition", "cb_sort", "assemble", "probe")
    ms_max = {k: S.max_over_ranks(float(ms[k]), dist, coll_dev) for k in cand}
    dom = max(cand, key=lambda k: ms_max[k])
    dom_bytes = S.sum_over_ranks(float(kern[dom].get("alg_bytes", 0)), dist, coll_dev)
    achieved = round(dom_bytes / (ms_max[dom] * 1e-3) / 1e9, 1) if ms_max[dom] > 0 else None
    peak = HBM_PEAK_GBS * world
    traffic = None
    if not var and os.path.exists(args.pmc):
        try:
            with open(args.pmc) as fh:
                pm = json.load(fh)
            traffic = pm.get("per_launch_hbm_bytes", {}).get(dom)
        except Exception:
            traffic = None
    ms_per_step = elapsed / args.steps * 1e3
    # the timed step minus its probe (launch gaps included); the stage pass's event-bracketed
    # build_total is reported beside it in `kernels`
    probe_ms = ms["probe"]
    build_ms = ms_per_step - probe_ms
    value = keys_all / (elapsed / args.steps) / 1e6
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "Mkeys/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": ("synthetic: variable-length 8-100 B keys (splitmix64), Zipf(0.99) probe mix, copied to HBM "
                 "before timing" if var else
                 "synthetic: sequential-id 24 B keys (filter_test format), generated in HBM"),
        "config": {"workload": wdesc, "filters_total": F_total,
                   "filters_per_gpu": F, "keys_per_filter": n, "key_len": "8-100" if var else 24,
                   "fingerprint_size": 26, "log_index_size": args.log_index_size, "seed": 42,
                   "parallelism": f"key-range shards, {world} rank(s), no data-path collective"},
        "build_mkeys_s": round(keys_all / (build_ms * 1e-3) / 1e6, 1),
        "probe_mkeys_s": round(S.sum_over_ranks(float(P), dist, coll_dev) / (probe_ms * 1e-3) / 1e6, 1),
        "e2e_pcie_mkeys_s": round(e2e, 1) if e2e else None,
        "e2e_pcie_serial_mkeys_s": round(e2e_serial, 1) if e2e else None,
        "e2e_pcie_hashes_mkeys_s": round(e2e_h, 1) if e2e_h else None,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": peak,
                     "unit": "GB/s", "frac": round(achieved / peak, 4) if achieved else None,
                     "traffic": traffic, "gpus": world,
                     "per_gpu_achieved": kern[dom].get("gbs"), "per_gpu_peak": HBM_PEAK_GBS,
                     "floor_ms": round(floor_ms, 4) if (floor_ms and dom == "probe") else None},
        # the probe's measured floor (ms per launch, slowest rank) and the probe's time over it
        "probe_floor": ({"floor_ms": round(floor_ms, 4), "probe_ms": round(probe_ms, 4),
                         "probe_over_floor": round(probe_ms / floor_ms, 3),
                         "what": "k_probe_floor: the probe's fast-path memory traffic (key staging, "
                                 "one 64-B line gather per probe, 8-B store) over the same runs, "
                                 "hash and decode removed"} if floor_ms else None),
        "kernels": kern,
        "build_total_stage_pass_ms": round(ms["build_total"], 4),
        "verified": verified,
        "sha_checked_filters": sha_checked,
    }
    if routed is not None:
        out["routed_probe"] = routed
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline_var(args, args.log_index_size, w, F, n) if var else \
            cpu_baseline(args, args.log_index_size, n)
        if cb is not None:
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu"] = round(value / cb["value"], 1)
            # device-resident GPU build against the all-core CPU hash + build (trunk semantics)
            out["build_speedup_vs_cpu"] = round(out["build_mkeys_s"] / cb["build_mkeys_s"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    batch.close()
    if dist is not None:
        dist.destroy_process_group()


def run_compaction(args, rank, world, dist, dev, coll_dev, backend):
    """Compaction chains (SURVEY.md §8(f) 'incremental adds'): the trunk grows a branch's
    filter by one routing_filter_add per compaction, merging the previous filter
    (src/trunk.c:3821-3835, src/routing_filter.c:355-368) and dropping it afterwards
    (routing_filter_dec_ref). Here F filters per GPU run CHAIN_ROUNDS such rounds in
    lockstep; round v of filter g adds keys (g << 32) + (v + 1) j, j < n, under value v --
    for g = 0 exactly tests/functional/filter_test.c:53-82. A round = create the batch (pooled
    device memory), build it from the device-resident keys with the previous round's
    batch as old filters, and release the superseded batch stream-ordered; the images stay
    in HBM (where the shim keeps them for lookups). One step = one whole chain; value = new
    keys / step time, whole job. Beside it (never as it): the same chain with every round's
    pages and index slots also read back into pinned host buffers (the clockcache pages'
    stand-in) on a copy stream, overlapping the next round's build -- PCIe-inclusive."""
    F = args.filters or WORKLOADS["compaction"][0]
    n = args.keys_per_filter or WORKLOADS["compaction"][1]
    V = CHAIN_ROUNDS
    g0 = rank * F
    cfg = E.routing_config_init(fingerprint_size=26, log_index_size=args.log_index_size, seed=42)
    eng = E.Engine(dev.index)
    stream = torch.cuda.Stream(device=dev)
    copy = torch.cuda.Stream(device=dev)
    st = stream.cuda_stream
    with torch.cuda.stream(stream):
        gid = torch.arange(g0, g0 + F, device=dev, dtype=torch.int64)[:, None] << 32
        j = torch.arange(n, device=dev, dtype=torch.int64)[None, :]
        keys = [K.ids_keys_torch((gid + (v + 1) * j).reshape(-1), 24) for v in range(V)]
        found = torch.empty(F * n, dtype=torch.int64, device=dev)
        del gid, j
    stream.synchronize()
    hp = hs = None

    def chain(readback, timing=False):
        """one chain of V rounds; returns (last batch, per-round wall ms, per-round build ms,
        per-round infos)"""
        prev = None
        walls, builds, infos_all = [], [], []
        evs = []
        for v in range(V):
            t0 = time.perf_counter()
            b = E.FilterBatch(cfg, [n] * F, [v] * F, old=[(prev, f) for f in range(F)] if prev else None,
                              engine=eng)
            if timing:
                b.set_timing(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            b.build_keys(keys[v], 24, stream=st)
            e1.record(stream)
            evs.append((e0, e1))
            if prev is not None:
                stream.wait_stream(copy)  # the previous round's read-back also reads prev
                prev.close(stream=st)
            inf = b.infos(stream=st)
            if readback:
                copy.wait_stream(stream)
                for f in range(F):
                    b.read_image_async(f, hp[f][: inf[f].num_pages * cfg.page_size], hs[f][: inf[f].num_indices],
                                       copy.cuda_stream)
            infos_all.append(inf)
            walls.append((time.perf_counter() - t0) * 1e3)
            prev = b
        copy.synchronize()
        stream.synchronize()
        builds = [a.elapsed_time(c) for a, c in evs]
        return prev, walls, builds, infos_all

    # sizing chain (untimed): the last round's filters are the largest
    last, _, _, inf0 = chain(False)
    last.close()
    hp = [torch.empty(i.num_pages * cfg.page_size, dtype=torch.uint8).pin_memory() for i in inf0[-1]]
    hs = [torch.empty(i.num_indices, dtype=torch.int64).pin_memory() for i in inf0[-1]]
    for _ in range(max(0, args.warmup)):
        last, *_ = chain(True)
        last.close()

    def barrier():
        if dist is not None:
            dist.barrier()

    steps = max(1, args.steps)
    walls, builds = np.zeros(V), np.zeros(V)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        last, w, bt, infos_all = chain(False)
        walls += w
        builds += bt
        if k + 1 < steps:
            last.close(stream=st)
    torch.cuda.synchronize()
    barrier()
    elapsed = S.max_over_ranks(time.perf_counter() - t0, dist, coll_dev)
    keys_job = S.sum_over_ranks(float(F * n * V), dist, coll_dev)
    walls /= steps
    builds /= steps
    last.close()

    # per-stage times of one chain's rounds (HIP events), outside the timed loop
    lastd, _, _, _ = chain(False, timing=True)
    stage_last = lastd.timings(0)
    lastd.close()

    # PCIe-inclusive chain (pages + slots read back every round), beside value
    rb_reps = 2
    rb_walls = np.zeros(V)
    torch.cuda.synchronize()
    tr = time.perf_counter()
    for k in range(rb_reps):
        last, w, _, infos_all = chain(True)
        rb_walls += w
        if k + 1 < rb_reps:
            last.close(stream=st)
    torch.cuda.synchronize()
    tr = S.max_over_ranks((time.perf_counter() - tr) / rb_reps, dist, coll_dev)
    rb_walls /= rb_reps

    # drop-in latency (beside value): one routing_filter_add of 2^20-1 host hashes through
    # rf_amd_filter_add -- what the shim pays per call -- fresh, then onto that filter
    dropin = None
    if rank == 0:
        hh = torch.empty(n, dtype=torch.int32, device=dev)
        E.hash_keys(cfg, keys[0][:n], 24, n, hh, engine=eng)
        h0 = hh.cpu().numpy().view(np.uint32).copy()
        E.hash_keys(cfg, keys[1][:n], 24, n, hh, engine=eng)
        h1 = hh.cpu().numpy().view(np.uint32).copy()
        E.routing_filter_add(cfg, None, h0, 0, engine=eng)  # warm
        t_f, t_i = [], []
        for _ in range(5):
            ta = time.perf_counter()
            f0 = E.routing_filter_add(cfg, None, h0, 0, engine=eng)
            tb = time.perf_counter()
            E.routing_filter_add(cfg, f0, h1, 1, engine=eng)
            tc = time.perf_counter()
            t_f.append(tb - ta)
            t_i.append(tc - tb)
        dropin = {"fresh_add_ms": round(float(np.median(t_f)) * 1e3, 3),
                  "incremental_add_ms": round(float(np.median(t_i)) * 1e3, 3),
                  "keys": n,
                  "note": "rf_amd_filter_add (host hashes in, host image out, old image uploaded), "
                          "median of 5"}
        del hh

    # ---- verification (outside the timed region) -------------------------------------
    # every round's keys find their value in the final filters (filter_test.c:100-116)
    ok = True
    counts = [n] * F
    for v in range(V):
        last.probe_keys_runs(keys[v], 24, counts, found, stream=st)
        stream.synchronize()
        ok = ok and bool((((found >> v) & 1) == 1).all().item())
    final = infos_all[-1]
    ok = ok and all(i.error == 0 and i.num_fingerprints == V * n for i in final)
    sha_checked = []
    if args.log_index_size == 8:
        with open(os.path.join(ROOT, "tests", "golden", "sha256.json")) as fh:
            gold = json.load(fh)
        for f in range(F):
            key = f"chain_f{g0 + f}_v{V}_n{n}_lis8"
            if key in gold:
                img = last.image(f)
                good = (hashlib.sha256(img.pages.tobytes()).hexdigest() == gold[key]["pages_sha256"] and
                        hashlib.sha256(img.slots.tobytes()).hexdigest() == gold[key]["slots_sha256"] and
                        final[f].num_unique == gold[key]["num_unique"])
                ok = ok and good
                sha_checked.append(g0 + f)
    # the read-back landed: the host copy of the last round equals the device image
    img0 = last.image(0)
    ok = ok and bool(np.array_equal(hp[0][: img0.pages.size].numpy(), img0.pages))
    last.close()
    verified = S.max_over_ranks(0.0 if ok else 1.0, dist, coll_dev) == 0.0

    # roofline of the dominant phase, the last round's incremental build: algorithmic bytes =
    # new keys (24 B) + the old filters' pages and slots read + the new pages and slots written
    pg = cfg.page_size
    old_b = sum(i.num_pages * pg + i.num_indices * 8 for i in infos_all[-2]) if V > 1 else 0
    new_b = sum(i.num_pages * pg + i.num_indices * 8 for i in final)
    alg = F * n * 24 + old_b + new_b
    b_ms = float(builds[-1])
    # job-wide: every rank's bytes over the slowest rank's build, against world x peak
    alg_all = S.sum_over_ranks(float(alg), dist, coll_dev)
    achieved = alg_all / (S.max_over_ranks(b_ms, dist, coll_dev) * 1e-3) / 1e9
    peak = HBM_PEAK_GBS * world
    readback_bytes = sum(i.num_pages * pg + i.num_indices * 8 for inf in infos_all for i in inf)
    ms_step = elapsed / steps * 1e3
    value = keys_job / (elapsed / steps) / 1e6
    out = {
        "metric": "routing_filter compaction chain: new keys/s through create + incremental build + release, device-resident",
        "value": round(value, 1), "unit": "Mkeys/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: filter_test-format 24 B keys (f << 32) + (v + 1) j, generated in HBM",
        "config": {"workload": WORKLOADS["compaction"][3], "filters_per_gpu": F, "rounds": V,
                   "keys_per_round": n, "fingerprints_final": V * n, "fingerprint_size": 26,
                   "log_index_size": args.log_index_size, "seed": 42,
                   "parallelism": f"filter shards, {world} rank(s), no data-path collective"},
        "round_wall_ms": [round(x, 3) for x in walls],
        "round_build_ms": [round(x, 3) for x in builds],
        "with_readback": {"mkeys_s": round(keys_job / tr / 1e6, 1), "chain_ms": round(tr * 1e3, 3),
                          "round_wall_ms": [round(x, 3) for x in rb_walls],
                          "readback_gb_per_chain": round(readback_bytes / 1e9, 3),
                          "readback_gbs": round(S.sum_over_ranks(readback_bytes, dist, coll_dev) / tr / 1e9, 1),
                          "note": "PCIe-inclusive: every round's pages and slots D2H into pinned host buffers"},
        "last_round_stages_ms": {k: round(v, 4) for k, v in stage_last.items() if k != "probe"},
        "roofline": {"bound": "hbm", "kernel": "incremental build (round 8, all stages)", "achieved": round(achieved, 1),
                     "peak": peak, "unit": "GB/s", "frac": round(achieved / peak, 4),
                     "traffic": None, "alg_bytes": int(alg_all), "gpus": world},
        "verified": verified, "sha_checked_filters": sha_checked,
        "num_unique_filter0": int(final[0].num_unique),
        "dropin_latency": dropin,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cpu_baseline as CB
        cb = CB.chain(args.log_index_size, V, n, threads=args.cpu_threads)
        if cb is not None:
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu"] = round(value / cb["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
