"""Multi-GPU sharding of environments.

Rank r of W owns global envs [r*N, (r+1)*N); every RNG stream is keyed by the
global env id, so per-env results do not depend on W. The only collective is a
tiny per-rollout reduction of episode statistics: each rank sums its env
partials in fixed env order, the partials are all-gathered (RCCL over xGMI on
GPUs, gloo on CPU) and summed in fixed rank order on every rank, which makes
the result bit-reproducible whatever ring/tree RCCL picks.
"""

from __future__ import annotations

import os


def shard(global_envs: int, world: int, rank: int) -> tuple[int, int]:
    """(env_offset, n_envs) of `rank` for an even split."""
    if global_envs % world:
        raise ValueError(f"{global_envs} envs do not split evenly over {world} ranks")
    n = global_envs // world
    return rank * n, n


def reduce_fixed_order(part, group=None):
    """A per-rank float64 partial -> the sum over ranks, the same bits on every rank: all_gather
    (RCCL over xGMI on GPUs, gloo on CPU) and a rank-order sum, whatever algorithm the collective
    picks. Without an initialised process group: the partial itself."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    if not dist.is_available() or not dist.is_initialized():
        return part
    world = dist.get_world_size(group)
    parts = [torch.zeros_like(part) for _ in range(world)]
    dist.all_gather(parts, part, group=group)
    total = parts[0].clone()
    for p in parts[1:]:
        total += p
    return total


def reduce_episode_stats(stats_local, group=None):
    """[n_local, 4] per-env statistics -> [4] float64 global sums (every rank)."""
    return reduce_fixed_order(stats_local.double().sum(0), group=group)


def dist_env() -> tuple[int, int, int]:
    """(rank, local_rank, world) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))
