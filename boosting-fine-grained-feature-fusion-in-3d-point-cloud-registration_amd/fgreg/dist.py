"""Multi-GPU: registration pairs are independent in eval, so the forward shards by pair.

One process per GPU (torchrun), no collective on the data path. The only exchange is
one all-gather of the per-pair results at the end of a batch (poses, (L, P, 3, 4) fp32
= 288 B per pair and layer stack), over RCCL/xGMI on MI355X ('nccl' backend) or gloo on
CPU. SURVEY.md §5 / §8(e): InstanceNorm is per cloud, Res2Net BatchNorm uses running
statistics in eval, attention and pose are per pair -- nothing couples the shards.
"""
from typing import List, Sequence

import torch
import torch.distributed as dist


def shard_range(n_pairs: int, world: int, rank: int):
    """Contiguous block of pairs for `rank` (equal-sized clouds, e.g. ModelNet)."""
    base, extra = divmod(n_pairs, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def balanced_shards(costs: Sequence[float], world: int) -> List[List[int]]:
    """Greedy longest-processing-time assignment of pairs to ranks (variable-size
    fragments, e.g. 3DMatch: cost ~ points per pair). Each shard keeps ascending order."""
    order = sorted(range(len(costs)), key=lambda i: -costs[i])
    load = [0.0] * world
    shards: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += costs[i]
    return [sorted(s) for s in shards]


def gather_pair_results(local: torch.Tensor, counts: Sequence[int], pair_dim: int = 1):
    """All-gather per-pair results whose pair axis is `pair_dim`; ranks may hold different
    numbers of pairs (`counts[r]`). Returns the concatenation in rank order."""
    world = dist.get_world_size()
    assert len(counts) == world
    if local.is_cuda and dist.get_backend() == 'gloo':     # gloo: exchange host copies
        return gather_pair_results(local.cpu(), counts, pair_dim).to(local.device)
    mx = max(counts)
    shape = list(local.shape)
    shape[pair_dim] = mx
    padded = local.new_zeros(shape)
    idx = [slice(None)] * local.dim()
    idx[pair_dim] = slice(0, local.shape[pair_dim])
    padded[tuple(idx)] = local
    bufs = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(bufs, padded.contiguous())
    parts = []
    for r in range(world):
        idx[pair_dim] = slice(0, counts[r])
        parts.append(bufs[r][tuple(idx)])
    return torch.cat(parts, dim=pair_dim)
