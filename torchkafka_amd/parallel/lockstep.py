"""Cross-rank lockstep for streaming DDP.

The reference has no notion of ranks: under torchrun every rank's consumers
would join one group and run at their own pace, so one rank running out of
records (or lagging) leaves the others hanging in the next gradient
all-reduce, and offsets committed by a fast rank describe a step the job as
a whole never finished.

:class:`Lockstep` makes every loader step a collective decision: each rank
contributes ``[have_batch, step, -step, commit_status]`` and one all-reduce(MIN)
tells all ranks whether *every* rank has a batch for this step (so they
continue or stop together), checks that they are on the same step and -- for
``commit='sync'``, where each rank commits batch k-1 BEFORE this agreement --
whether every rank's commit went through (2 stored, 1 a CommitFailedError was
logged and swallowed, 0 a commit raised: every rank raises).  Because the
collective completes only when every rank has reached step k, it is also the
barrier after which batch k-1's offsets are committed on every rank.

On ROCm the ``nccl`` backend is RCCL: the 24-byte all-reduce rides xGMI and is
latency-bound, so it is issued on a private side stream (never behind the
user's queued compute) and read back through pinned memory.  With ``gloo``
(CPU tests) the same code runs on host tensors.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class LockstepError(RuntimeError):
    pass


class Lockstep:
    """``transport``: a node-local shared-memory transport (``_tkcore.ShmLockstep``, see
    ``csrc/core/shm_lockstep.h``) to agree through instead of the group's all-reduce."""

    def __init__(self, group=None, device: torch.device | None = None, transport=None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("Lockstep needs an initialised torch.distributed process group")
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.transport = transport
        backend = dist.get_backend(group)
        self.on_device = backend == "nccl" and transport is None
        if self.on_device:
            if device is None or device.type != "cuda":
                device = torch.device("cuda", torch.cuda.current_device())
            self.device = device
            self._stream = torch.cuda.Stream(device=device)
            self._dev = torch.zeros(4, dtype=torch.int64, device=device)
            self._h_in = torch.zeros(4, dtype=torch.int64).pin_memory()
            self._h_out = torch.zeros(4, dtype=torch.int64).pin_memory()
        else:
            self.device = torch.device("cpu")
            self._buf = torch.zeros(4, dtype=torch.int64)
        self.collectives = 0
        self.group_commit_status = 2
        self.group_commit_failures = 0

    def _allreduce_min(self, *w: int) -> tuple[int, ...]:
        self.collectives += 1
        if self.transport is not None:
            try:
                return tuple(self.transport.allreduce_min(*w))
            except RuntimeError as e:
                raise LockstepError(str(e)) from e
        if not self.on_device:
            for i, v in enumerate(w):
                self._buf[i] = v
            dist.all_reduce(self._buf, op=dist.ReduceOp.MIN, group=self.group)
            return tuple(int(v) for v in self._buf.tolist())
        for i, v in enumerate(w):
            self._h_in[i] = v
        with torch.cuda.stream(self._stream):
            self._dev.copy_(self._h_in, non_blocking=True)
            dist.all_reduce(self._dev, op=dist.ReduceOp.MIN, group=self.group)
            self._h_out.copy_(self._dev, non_blocking=True)
        self._stream.synchronize()
        return tuple(int(v) for v in self._h_out.tolist())

    def agree(self, have_batch: bool, step: int, commit_status: int = 2) -> bool:
        """True iff every rank has a batch for ``step``.  Raises if ranks disagree on the step, or
        if some rank's commit raised (``commit_status`` 0 anywhere)."""
        have, lo, neg_hi, status = self._allreduce_min(1 if have_batch else 0, step, -step, commit_status)
        if lo != -neg_hi:
            raise LockstepError(f"ranks are out of step: min step {lo}, max step {-neg_hi} (this rank: {step})")
        self.group_commit_status = status
        if status == 1:
            self.group_commit_failures += 1
        if status <= 0:
            raise LockstepError(f"lockstep: a rank's commit before step {step} failed; every rank stops here")
        return bool(have)

    def barrier(self, commit_status: int = 2) -> None:
        status = self._allreduce_min(0, 0, 0, commit_status)[3]
        if status <= 0:
            raise LockstepError("lockstep: a rank's last commit failed")
