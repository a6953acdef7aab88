"""Deterministic partition sharding across DDP ranks and loader workers.

The reference leaves partition ownership to Kafka's group assignor: every
DataLoader worker is an independent group member with identical kwargs
(kafka_dataset.py:38-39, 219-231; B21) and the assignment changes at every
rebalance.  For a multi-GPU job that is unusable: ranks would not know which
data they own, and a worker joining late rebalances everyone.  The static
map below is stable, needs no coordination, and spreads partitions so that
rank r of W sees every W-th partition (p % W == r) and, inside a rank, the
workers take turns ((p // W) % num_workers == worker).
"""
from __future__ import annotations


def shard_partitions(n_partitions: int, rank: int = 0, world_size: int = 1, worker_id: int = 0,
                     num_workers: int = 1) -> list[int]:
    if world_size < 1 or num_workers < 1:
        raise ValueError("world_size and num_workers must be >= 1")
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside [0, {world_size})")
    if not 0 <= worker_id < num_workers:
        raise ValueError(f"worker_id {worker_id} outside [0, {num_workers})")
    return [p for p in range(n_partitions)
            if p % world_size == rank and (p // world_size) % num_workers == worker_id]


def shard_owner(partition: int, world_size: int = 1, num_workers: int = 1) -> tuple[int, int]:
    """(rank, worker) owning ``partition``."""
    return partition % world_size, (partition // world_size) % num_workers


def dist_rank_world() -> tuple[int, int]:
    """Rank/world from an initialised torch.distributed group, else the torchrun env, else (0, 1)."""
    import os

    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except Exception:  # noqa: BLE001
        pass
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
