"""Routed probes across ranks (splinterdb_amd/route.py, rf_amd_route_probes & co.).

CPU: the ProbeRouter's exchange (counts, pairs, results: three all-to-alls under gloo,
world 2 and 3) with a numpy restatement of the routing kernels and oracle filters as the
owners' probe; every probe's found_values must equal a direct lookup in its filter.
GPU: the partition kernel against a numpy stable partition (ragged sizes, world 1-16, bad
ids), unroute, and the router end to end on cuda:0 (world 1, and 2 gloo ranks sharing
the device) against the oracle."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from splinterdb_amd import keys as K
from splinterdb_amd import route as R
from splinterdb_amd import shard as S


def _np_partition(h, gfid, route, world):
    """Stable partition of probes by owner rank: (pairs, perm, counts)."""
    dest = (route[gfid] & 0xFF).astype(np.int64)
    perm = np.argsort(dest, kind="stable")
    lid = (route[gfid] >> 8).astype(np.uint64)
    pairs = (lid << np.uint64(32)) | h.astype(np.uint64)
    return pairs[perm], perm.astype(np.uint32), np.bincount(dest, minlength=world).tolist()


class NumpyRouteOps:
    """CPU restatement of the routing kernels; the owner's probe is the oracle."""

    def scratch_bytes(self, n, world):
        return 16

    def route(self, d_hashes, d_gfid, n, d_route, num_filters, world, d_pairs, d_perm, d_scratch):
        h = d_hashes[:n].numpy().view(np.uint32)
        g = d_gfid[:n].numpy().view(np.uint32)
        assert (g < num_filters).all()
        pairs, perm, counts = _np_partition(h, g, d_route.numpy().view(np.uint32), world)
        d_pairs[:n] = torch.from_numpy(pairs.view(np.int64))
        d_perm[:n] = torch.from_numpy(perm.view(np.int32))
        return counts

    def probe(self, filters, d_pairs, m, d_found):
        p = d_pairs[:m].numpy().view(np.uint64)
        lid, h = (p >> np.uint64(32)).astype(np.int64), (p & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        out = np.zeros(m, dtype=np.uint64)
        for f in np.unique(lid):
            sel = lid == f
            out[sel] = filters[f].lookup_hashes(h[sel])
        d_found[:m] = torch.from_numpy(out.view(np.int64))

    def unroute(self, d_back, d_perm, n, d_found):
        perm = d_perm[:n].numpy().view(np.uint32).astype(np.int64)
        d_found[torch.from_numpy(perm)] = d_back[:n]


def test_route_table():
    sh = S.plan_shards(7, 100, 3)
    t = R.route_table(sh)
    assert t.tolist() == [0 << 8 | 0, 1 << 8 | 0, 2 << 8 | 0, 0 << 8 | 1, 1 << 8 | 1, 0 << 8 | 2, 1 << 8 | 2]


def _probe_set(rng, F, n, P):
    """P probes over all F filters: half inserted keys (filter f holds ids [f*n, (f+1)*n)),
    half random ids; the probe's filter is the key range its id falls in (or random)."""
    ids = np.concatenate([rng.integers(0, F * n, size=P // 2), rng.integers(F * n, 4 * F * n, size=P - P // 2)])
    gfid = np.where(ids < F * n, ids // n, rng.integers(0, F, size=P)).astype(np.uint32)
    return ids.astype(np.uint64), gfid


def _cpu_worker(rank, world, port, F, n, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    cfg = O.make_config()
    shards = S.plan_shards(F, n, world)
    me = shards[rank]
    mine = [O.filter_add(cfg, O.hash_fixed(K.seq_keys(f * n, n).reshape(-1), 24), value=f % 8)
            for f in range(me.filter_begin, me.filter_end)]
    router = R.ProbeRouter(shards, rank, mine, "cpu", dist=dist, coll_device="cpu", ops=NumpyRouteOps())
    rng = np.random.default_rng(100 + rank)
    ids, gfid = _probe_set(rng, F, n, 3000 + 517 * rank)
    h = O.hash_fixed(np.concatenate([K.seq_keys(int(i), 1) for i in ids]).reshape(-1), 24)
    found = torch.zeros(len(ids), dtype=torch.int64)
    send, recv = router.lookup_hashes(torch.from_numpy(h.view(np.int32)), torch.from_numpy(gfid.view(np.int32)),
                                      len(ids), found)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), h=h, gfid=gfid, found=found.numpy(), send=send, recv=recv)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_router_gloo_matches_direct_lookup(oracle, world):
    F, n = 5, 3000
    port = 29700 + world * 10 + (os.getpid() % 500)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_cpu_worker, args=(world, port, F, n, d), nprocs=world, join=True)
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    cfg = oracle.make_config()
    flt = [oracle.filter_add(cfg, oracle.hash_fixed(K.seq_keys(f * n, n).reshape(-1), 24), value=f % 8)
           for f in range(F)]
    for r in range(world):
        h, gfid, found = res[r]["h"], res[r]["gfid"], res[r]["found"].view(np.uint64)
        for f in range(F):
            sel = gfid == f
            assert (found[sel] == flt[f].lookup_hashes(h[sel])).all(), (r, f)
        # what rank r sent to q is what q received from r
        for q in range(world):
            assert res[r]["send"][q] == res[q]["recv"][r]


# ---------------------------------------------------------------------------- GPU --------
def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("n,world,F", [(0, 2, 4), (1, 1, 1), (1000, 3, 7), (16384, 8, 8), (16385, 5, 9),
                                       (100003, 16, 40), (250000, 8, 1024)])
def test_route_kernel_matches_stable_partition(n, world, F):
    from splinterdb_amd import engine as E
    rng = np.random.default_rng(n + world)
    route = R.route_table(S.plan_shards(F, 10, world))
    h = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    g = rng.integers(0, F, size=n).astype(np.uint32)
    if n > 100:  # skewed: most probes to one filter
        g[rng.random(n) < 0.5] = F - 1
    pairs = torch.zeros(max(n, 1), dtype=torch.int64, device="cuda:0")
    perm = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda:0")
    scratch = torch.zeros(E.route_scratch_bytes(n, world), dtype=torch.uint8, device="cuda:0")
    counts = E.route_probes(_dev(h.view(np.int32)) if n else pairs, _dev(g.view(np.int32)) if n else pairs, n,
                            _dev(route.view(np.int32)), F, world, pairs, perm, scratch)
    torch.cuda.synchronize()
    ep, eperm, ec = _np_partition(h, g, route, world)
    assert counts == ec
    assert (pairs.cpu().numpy().view(np.uint64)[:n] == ep).all()
    assert (perm.cpu().numpy().view(np.uint32)[:n] == eperm).all()
    # unroute inverts the permutation
    back = torch.from_numpy(np.arange(n, dtype=np.int64) * 3 + 1).to("cuda:0") if n else pairs
    out = torch.zeros(max(n, 1), dtype=torch.int64, device="cuda:0")
    E.unroute_found(back, perm, n, out)
    torch.cuda.synchronize()
    exp = np.zeros(n, dtype=np.int64)
    exp[eperm.astype(np.int64)] = np.arange(n, dtype=np.int64) * 3 + 1
    assert (out.cpu().numpy()[:n] == exp).all()


@pytest.mark.gpu
def test_route_rejects_bad_ids():
    from splinterdb_amd import engine as E
    n, F, world = 5000, 4, 2
    route = R.route_table(S.plan_shards(F, 10, world))
    g = np.zeros(n, dtype=np.uint32)
    g[1234] = F  # out of range
    buf = lambda dt: torch.zeros(n, dtype=dt, device="cuda:0")  # noqa: E731
    scratch = torch.zeros(E.route_scratch_bytes(n, world), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(E.PlatformStatusError):
        E.route_probes(buf(torch.int32), _dev(g.view(np.int32)), n, _dev(route.view(np.int32)), F, world,
                       buf(torch.int64), buf(torch.int32), scratch)
    bad = route.copy()
    bad[2] = (bad[2] & ~np.uint32(0xFF)) | np.uint32(world)  # rank >= world
    g[1234] = 2
    with pytest.raises(E.PlatformStatusError):
        E.route_probes(buf(torch.int32), _dev(g.view(np.int32)), n, _dev(bad.view(np.int32)), F, world,
                       buf(torch.int64), buf(torch.int32), scratch)
    with pytest.raises(E.PlatformStatusError):
        E.route_probes(buf(torch.int32), buf(torch.int32), n, _dev(route.view(np.int32)), F, 17,
                       buf(torch.int64), buf(torch.int32), scratch)


def _gpu_rank(rank, world, F, n, cfg, dist=None, coll_device=None):
    """Build this rank's shard on cuda:0, route probes over all F filters, return arrays."""
    from oracle import oracle as O
    from splinterdb_amd import engine as E
    shards = S.plan_shards(F, n, world)
    me = shards[rank]
    vals = [f % 8 for f in range(me.filter_begin, me.filter_end)]
    b = E.FilterBatch(cfg, [n] * me.num_filters, vals)
    kk = K.seq_keys(me.filter_begin * n, me.num_filters * n).reshape(-1)
    b.build_keys(_dev(kk), 24)
    router = R.ProbeRouter(shards, rank, b, "cuda:0", dist=dist, coll_device=coll_device)
    rng = np.random.default_rng(7 + rank)
    ids, gfid = _probe_set(rng, F, n, 20000 + 333 * rank)
    keys = np.concatenate([K.seq_keys(int(i), 1) for i in ids]).reshape(-1)
    h = O.hash_fixed(keys, 24)
    d_h = torch.zeros(len(ids), dtype=torch.int32, device="cuda:0")
    E.hash_keys(cfg, _dev(keys), 24, len(ids), d_h)
    found = torch.zeros(len(ids), dtype=torch.int64, device="cuda:0")
    router.lookup_hashes(d_h, _dev(gfid.view(np.int32)), len(ids), found)
    torch.cuda.synchronize()
    assert (d_h.cpu().numpy().view(np.uint32) == h).all()
    return h, gfid, found.cpu().numpy().view(np.uint64)


def _check_against_oracle(oracle, F, n, h, gfid, found):
    cfg = oracle.make_config()
    for f in range(F):
        flt = oracle.filter_add(cfg, oracle.hash_fixed(K.seq_keys(f * n, n).reshape(-1), 24), value=f % 8)
        sel = gfid == f
        assert (found[sel] == flt.lookup_hashes(h[sel])).all(), f


@pytest.mark.gpu
def test_router_world1_gpu(oracle):
    from splinterdb_amd import engine as E
    F, n = 4, 50000
    h, gfid, found = _gpu_rank(0, 1, F, n, E.routing_config_init())
    _check_against_oracle(oracle, F, n, h, gfid, found)


def _gpu_worker(rank, world, port, F, n, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splinterdb_amd import engine as E
    h, gfid, found = _gpu_rank(rank, world, F, n, E.routing_config_init(), dist=dist, coll_device="cpu")
    np.savez(os.path.join(outdir, f"g{rank}.npz"), h=h, gfid=gfid, found=found)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_router_two_ranks_on_one_gpu(oracle):
    """Two processes share cuda:0; the exchange runs over gloo (RCCL needs one GPU per rank)."""
    F, n, world = 5, 40000, 2
    port = 29900 + (os.getpid() % 500)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gpu_worker, args=(world, port, F, n, d), nprocs=world, join=True)
        for r in range(world):
            z = np.load(os.path.join(d, f"g{r}.npz"))
            _check_against_oracle(oracle, F, n, z["h"], z["gfid"], z["found"])


# ---- replicated probes: export / all-gather / import -------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("device_resident", [True, False])
def test_export_import_round_trip(oracle, device_resident):
    from splinterdb_amd import engine as E
    cfg = E.routing_config_init()
    sizes, vals = [30000, 1, 250000, 4097], [3, 0, 7, 1]
    b = E.FilterBatch(cfg, sizes, vals)
    kk = K.seq_keys(0, sum(sizes)).reshape(-1)
    b.build_keys(_dev(kk), 24)
    infos, pbytes, nslots = b.export_sizes()
    d_p = torch.zeros(pbytes, dtype=torch.uint8, device="cuda:0")
    d_s = torch.zeros(nslots, dtype=torch.int64, device="cuda:0")
    b.export(d_p, d_s)
    torch.cuda.synchronize()
    src_p, src_s = (d_p, d_s) if device_resident else (d_p.cpu().numpy(), d_s.cpu().numpy())
    imp = E.FilterBatch.imported(cfg, infos, src_p, src_s, device_resident=device_resident)
    for f in range(len(sizes)):
        a, c = b.image(f), imp.image(f)
        assert (a.num_unique, a.num_pages) == (c.num_unique, c.num_pages)
        assert (a.pages == c.pages).all() and (a.slots == c.slots).all()
    rng = np.random.default_rng(5)
    P = 50000
    ids = rng.integers(0, 2 * sum(sizes), size=P).astype(np.uint64)
    fid = rng.integers(0, len(sizes), size=P).astype(np.uint32)
    pk = _dev(K.ids_keys(ids).reshape(-1))
    f1 = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    f2 = torch.zeros(P, dtype=torch.int64, device="cuda:0")
    b.probe_keys(pk, 24, _dev(fid.view(np.int32)), P, f1)
    imp.probe_keys(pk, 24, _dev(fid.view(np.int32)), P, f2)
    torch.cuda.synchronize()
    assert torch.equal(f1, f2)
    with pytest.raises(E.PlatformStatusError):  # geometry that no build produces
        bad = E.RfFilterInfo(infos[0].num_fingerprints, 1, 0, infos[0].num_indices * 2, infos[0].num_pages, 0)
        E.FilterBatch.imported(cfg, [bad], d_p, d_s)


def _replica_worker(rank, world, port, F, n, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from splinterdb_amd import engine as E
    cfg = E.routing_config_init()
    me = S.plan_shards(F, n, world)[rank]
    b = E.FilterBatch(cfg, [n] * me.num_filters, [f % 8 for f in range(me.filter_begin, me.filter_end)])
    b.build_keys(_dev(K.seq_keys(me.filter_begin * n, me.num_filters * n).reshape(-1)), 24)
    rep = R.replicate_images(b, world, "cuda:0", dist=dist, coll_device="cpu")
    assert rep.F == F
    rng = np.random.default_rng(11 + rank)
    ids, gfid = _probe_set(rng, F, n, 30000)
    keys = np.concatenate([K.seq_keys(int(i), 1) for i in ids]).reshape(-1)
    found = torch.zeros(len(ids), dtype=torch.int64, device="cuda:0")
    rep.probe_keys(_dev(keys), 24, _dev(gfid.view(np.int32)), len(ids), found)
    torch.cuda.synchronize()
    np.savez(os.path.join(outdir, f"p{rank}.npz"), h=O.hash_fixed(keys, 24), gfid=gfid,
             found=found.cpu().numpy().view(np.uint64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_replicated_images_two_ranks(oracle):
    F, n, world = 5, 30000, 2
    port = 30400 + (os.getpid() % 500)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_replica_worker, args=(world, port, F, n, d), nprocs=world, join=True)
        for r in range(world):
            z = np.load(os.path.join(d, f"p{r}.npz"))
            _check_against_oracle(oracle, F, n, z["h"], z["gfid"], z["found"])
