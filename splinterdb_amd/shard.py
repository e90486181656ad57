"""Key-range sharding of filter batches across GPUs (one process per GPU).

SplinterDB builds one routing filter per trunk pivot, i.e. per key range
(src/trunk.c:4133-4170, one bundle compaction per pivot), and the builds are independent.
So the multi-GPU layout is a partition of the filters into contiguous ranges, one range
per rank: no exchange on the data path (weak scaling for the per-GPU C2 workload, strong
scaling for the fixed-size C4 workload). torch.distributed (RCCL over xGMI on the GPU box,
gloo in the CPU tests) is used only for the start/stop barrier and the max-over-ranks
timing reduction.
"""
from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    filter_begin: int  # first global filter id owned by this rank
    filter_end: int    # one past the last
    key_begin: int     # first global key id (contiguous key ranges per filter)
    key_end: int

    @property
    def num_filters(self):
        return self.filter_end - self.filter_begin

    @property
    def num_keys(self):
        return self.key_end - self.key_begin


def plan_shards(num_filters: int, keys_per_filter: int, world: int):
    """Contiguous, balanced filter ranges: rank r owns filters [b_r, e_r) and their keys."""
    if world < 1 or num_filters < 1:
        raise ValueError("need world >= 1 and num_filters >= 1")
    q, r = divmod(num_filters, world)
    shards, b = [], 0
    for rank in range(world):
        e = b + q + (1 if rank < r else 0)
        shards.append(Shard(rank, world, b, e, b * keys_per_filter, e * keys_per_filter))
        b = e
    return shards


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """The bench contract's timing: max over ranks (identity when not distributed)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, dist=None, device=None) -> float:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
