"""Multi-process (gloo, CPU) tests of the key-range sharding used by bench.py --gpus N.

The data path has no collective; what must hold is that the per-rank shards partition the
filters / key ranges exactly, that every rank can build its shard's filters independently
with results identical to a single-process build (checked here with the oracle as the
stand-in worker, on CPU), and that timing is reduced with MAX over ranks."""
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from splinterdb_amd import keys as K
from splinterdb_amd import shard as S


@pytest.mark.parametrize("F,world", [(8, 1), (8, 2), (1024, 8), (7, 3), (3, 4)])
def test_plan_shards_partitions(F, world):
    n = 1000
    sh = S.plan_shards(F, n, world)
    assert len(sh) == world
    assert sh[0].filter_begin == 0 and sh[-1].filter_end == F
    for a, b in zip(sh, sh[1:]):
        assert a.filter_end == b.filter_begin and a.key_end == b.key_begin
    sizes = [s.num_filters for s in sh]
    assert max(sizes) - min(sizes) <= 1
    assert sum(s.num_keys for s in sh) == F * n


def _worker(rank, world, port, F, n, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    me = S.plan_shards(F, n, world)[rank]
    cfg = O.make_config()
    res = []
    for f in range(me.filter_begin, me.filter_end):
        h = O.hash_fixed(K.seq_keys(f * n, n).reshape(-1), 24)
        flt = O.filter_add(cfg, h)
        res.append((f, flt.num_unique, flt.num_pages, int(flt.pages().sum(dtype=np.uint64))))
    # timing contract: max over ranks
    t = S.max_over_ranks(float(rank + 1), dist)
    total = S.sum_over_ranks(float(me.num_keys), dist)
    np.save(os.path.join(outdir, f"r{rank}.npy"), np.array(res, dtype=np.int64))
    np.save(os.path.join(outdir, f"t{rank}.npy"), np.array([t, total]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_match_single_process(oracle):
    F, n, world = 6, 20000, 2
    port = 29500 + (os.getpid() % 1000)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, port, F, n, d), nprocs=world, join=True)
        got = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)])
        times = [np.load(os.path.join(d, f"t{r}.npy")) for r in range(world)]
    assert sorted(got[:, 0].tolist()) == list(range(F))
    cfg = oracle.make_config()
    for f, nu, npg, csum in got:
        flt = oracle.filter_add(cfg, oracle.hash_fixed(K.seq_keys(f * n, n).reshape(-1), 24))
        assert (nu, npg, int(flt.pages().sum(dtype=np.uint64))) == (flt.num_unique, flt.num_pages, csum)
    for t, total in times:
        assert t == float(world) and total == float(F * n)
