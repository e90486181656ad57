"""Routed probes across ranks: the serving side of the key-range sharding.

Builds shard by key range with no exchange (shard.py). A lookup, though, arrives on
whichever rank serves the request: in SplinterDB a point lookup consults the routing filter
of the trunk node owning the key's range (src/trunk.c:6008-6075). With filters spread over
ranks, probes must move to the owning rank and the found_values bit-vectors come back:
one all-to-all each way (RCCL over xGMI on the GPU box; gloo in the CPU tests).

The alternative when lookups are frequent and filters change rarely: replicate the images
once (replicate_images: one all-gather of every rank's packed pages + slots, imported on
each rank as a probe-only batch of all filters) and probe locally with no per-lookup
exchange.

Per lookup batch on every rank (routed):
  1. hash the keys where they are (XXH32, rf_amd_hash_keys): 4 B instead of the key moves;
  2. rf_amd_route_probes: stable partition of (hash, local filter id) pairs by owner rank,
     with per-rank counts (the all-to-all split sizes);
  3. all_to_all of the counts, then of the pairs;
  4. the owner probes the pairs it received against its own batch (k_probe, pair input);
  5. reverse all_to_all of the found_values;
  6. rf_amd_unroute_found puts each result back at its probe's position.
"""
import numpy as np

from . import engine as E


def route_table(shards):
    """route[g] = local filter id << 8 | owning rank, for every global filter id g."""
    t = np.zeros(shards[-1].filter_end, dtype=np.uint32)
    for sh in shards:
        g = np.arange(sh.filter_begin, sh.filter_end, dtype=np.uint32)
        t[g] = ((g - sh.filter_begin) << 8) | sh.rank
    return t


class GpuRouteOps:
    """The device kernels behind ProbeRouter (the C ABI's rf_amd_route_probes & co.)."""

    def __init__(self, engine=None):
        self.engine = engine

    def scratch_bytes(self, n, world):
        return E.route_scratch_bytes(n, world)

    def route(self, d_hashes, d_gfid, n, d_route, num_filters, world, d_pairs, d_perm, d_scratch):
        return E.route_probes(d_hashes, d_gfid, n, d_route, num_filters, world, d_pairs, d_perm, d_scratch,
                              engine=self.engine)

    def probe(self, batch, d_pairs, m, d_found):
        batch.probe_pairs(d_pairs, m, d_found)

    def unroute(self, d_back, d_perm, n, d_found):
        E.unroute_found(d_back, d_perm, n, d_found, engine=self.engine)


class ProbeRouter:
    """Routes probes (hash, global filter id) to the ranks owning the filters.

    shards: shard.plan_shards(...) (the same on every rank); batch: this rank's FilterBatch
    (its filters in global order, local id = global id - filter_begin). coll_device is
    where the collectives run: the GPU under RCCL, "cpu" under gloo (rehearsal/tests).
    collective_at_one: run the all-to-alls through `dist` with one rank too (the RCCL path of
    a multi-GPU run, exercised on one GPU), instead of a local copy.
    """

    def __init__(self, shards, rank, batch, device, dist=None, coll_device=None, ops=None,
                 collective_at_one=False):
        import torch
        self.torch = torch
        self.shards, self.rank, self.batch = shards, rank, batch
        self.world = len(shards)
        if not 1 <= self.world <= E.ROUTE_MAX_WORLD:
            raise ValueError(f"routed probes support 1..{E.ROUTE_MAX_WORLD} ranks")
        self.num_filters = shards[-1].filter_end
        self.device = torch.device(device)
        self.dist = dist
        self.coll_device = torch.device(coll_device) if coll_device is not None else self.device
        self.ops = ops or GpuRouteOps()
        self.local = self.world == 1 and not (collective_at_one and dist is not None)
        self.d_route = torch.from_numpy(route_table(shards).view(np.int32)).to(self.device)
        self._cap = -1

    def _buffers(self, n):
        if n > self._cap:
            t = self.torch
            cap = max(n, 1)
            self.d_pairs = t.empty(cap, dtype=t.int64, device=self.device)
            self.d_perm = t.empty(cap, dtype=t.int32, device=self.device)
            self.d_scratch = t.empty(self.ops.scratch_bytes(cap, self.world), dtype=t.uint8, device=self.device)
            self._cap = n

    def _a2a(self, out, inp, out_splits, in_splits):
        """all_to_all_single on the collective device (copies through it under gloo)."""
        t = self.torch
        if self.local:
            out.copy_(inp)
            return
        if self.coll_device == out.device and self.coll_device == inp.device:
            self.dist.all_to_all_single(out, inp, out_splits, in_splits)
            return
        o = t.empty(out.shape, dtype=out.dtype, device=self.coll_device)
        self.dist.all_to_all_single(o, inp.to(self.coll_device), out_splits, in_splits)
        out.copy_(o)

    def lookup_hashes(self, d_hashes, d_gfid, n, d_found):
        """found_values of n probes (XXH32 hashes + global filter ids) into d_found (int64)."""
        t = self.torch
        self._buffers(n)
        send = self.ops.route(d_hashes, d_gfid, n, self.d_route, self.num_filters, self.world,
                              self.d_pairs, self.d_perm, self.d_scratch)
        if self.local:
            recv = list(send)
        else:
            sc = t.tensor(send, dtype=t.int64, device=self.coll_device)
            rc = t.empty(self.world, dtype=t.int64, device=self.coll_device)
            self.dist.all_to_all_single(rc, sc)
            recv = [int(x) for x in rc.tolist()]
        m = sum(recv)
        pairs_in = t.empty(max(m, 1), dtype=t.int64, device=self.device)
        self._a2a(pairs_in[:m], self.d_pairs[:n], recv, send)
        found_local = t.zeros(max(m, 1), dtype=t.int64, device=self.device)
        if m:
            self.ops.probe(self.batch, pairs_in, m, found_local)
        back = t.empty(max(n, 1), dtype=t.int64, device=self.device)
        self._a2a(back[:n], found_local[:m], send, recv)
        if n:
            self.ops.unroute(back, self.d_perm, n, d_found)
        return send, recv


_INFO_FIELDS = ("num_fingerprints", "num_unique", "value_size", "num_indices", "num_pages", "error")


def _all_gather_padded(dist, t, world):
    """all_gather of 1-D tensors of different lengths (padded to the longest)."""
    import torch
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    m = max(max(ns), 1)
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return [o[:k] for o, k in zip(outs, ns)]


def replicate_images(batch, world, device, dist=None, coll_device=None, engine=None, collective_at_one=False):
    """Every rank's filters (in rank = global filter order) as one probe-only batch on this
    rank: pack (rf_amd_batch_export), all-gather pages, slots and filter infos, import
    (rf_amd_batch_import). Probes then use global filter ids locally. collective_at_one: run
    the all-gathers at world size 1 too (tests: the RCCL path on one GPU)."""
    import torch
    device = torch.device(device)
    coll = torch.device(coll_device) if coll_device is not None else device
    infos, pbytes, nslots = batch.export_sizes()
    d_pages = torch.empty(max(pbytes, 1), dtype=torch.uint8, device=device)
    d_slots = torch.empty(max(nslots, 1), dtype=torch.int64, device=device)
    batch.export(d_pages, d_slots)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    d_pages, d_slots = d_pages[:pbytes], d_slots[:nslots]
    inf = torch.tensor([[getattr(i, k) for k in _INFO_FIELDS] for i in infos], dtype=torch.int64).reshape(-1)
    if world == 1 and not collective_at_one:
        parts = [(inf, d_pages, d_slots)]
    else:
        gi = _all_gather_padded(dist, inf.to(coll), world)
        gp = _all_gather_padded(dist, d_pages.to(coll), world)
        gs = _all_gather_padded(dist, d_slots.to(coll), world)
        parts = list(zip(gi, gp, gs))
    all_inf = torch.cat([p[0].cpu() for p in parts]).reshape(-1, len(_INFO_FIELDS)).tolist()
    rinfos = [E.RfFilterInfo(*[int(x) for x in row]) for row in all_inf]
    pages = torch.cat([p[1] for p in parts])
    slots = torch.cat([p[2] for p in parts])
    on_dev = pages.device.type == "cuda"
    return E.FilterBatch.imported(batch.cfg, rinfos, pages, slots, device_resident=on_dev,
                                  engine=engine or batch.engine)

