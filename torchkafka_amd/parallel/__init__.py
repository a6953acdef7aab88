"""Multi-rank support: static partition sharding and the RCCL commit lockstep."""
from .sharding import dist_rank_world, shard_owner, shard_partitions

__all__ = ["shard_partitions", "shard_owner", "dist_rank_world", "Lockstep"]


def __getattr__(name):
    if name in ("Lockstep", "LockstepError"):
        from . import lockstep

        return getattr(lockstep, name)
    raise AttributeError(name)
