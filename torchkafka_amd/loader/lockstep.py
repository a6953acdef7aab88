"""DeviceLoader's cross-rank lockstep: which transport agrees on every step, the native RCCL
communicator, and the stream plan against the process's hardware queues.

The reference commits per batch with no agreement between ranks (/root/reference/src/
auto_commit.py:55-58); here every rank's step k is agreed before it is delivered and committed
(``csrc/core/lockstep.h``), over RCCL on GPUs or the process group's all-reduce otherwise.
"""
from __future__ import annotations

import os

import torch

from ..ops.native import hip


def _host_allreduce_min(group):
    """all-reduce(MIN) of the lockstep's four int64 words (credit, step, -step, commit status) over a
    CPU (gloo) group, for the driver's PyLockstep transport."""
    import torch.distributed as dist

    if dist.get_backend(group) != "gloo":
        group = dist.new_group(backend="gloo")  # collective: every rank builds its loader iterator
    buf = torch.zeros(4, dtype=torch.int64)

    def allreduce_min(a: int, b: int, c: int, d: int):
        buf[0], buf[1], buf[2], buf[3] = a, b, c, d
        dist.all_reduce(buf, op=dist.ReduceOp.MIN, group=group)
        return int(buf[0]), int(buf[1]), int(buf[2]), int(buf[3])

    return allreduce_min


def _host_key() -> str:
    """What identifies this host to the other ranks: hostname and the kernel's boot id (two
    containers of one machine share /dev/shm only if they share the boot and the IPC namespace;
    the segment's attach check catches the rest)."""
    import socket

    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return f"{socket.gethostname()}/{boot}"


class LoaderLockstep:
    """Mixin of :class:`~torchkafka_amd.loader.DeviceLoader`: ``lockstep``, ``lockstep_depth``,
    ``lockstep_commit_every``, ``lockstep_timeout``, ``world_size``, ``device``, ``native``, ``plan``,
    the live ``_run``."""

    def _lockstep_depth(self, transport) -> int:
        """Tuning.lockstep_depth, or its auto value: an RCCL agreement takes ~60-180 µs to come back
        while device-decoded steps take ~5 µs, so with the 64-deep ring the next one is issued 32
        steps before the credits run out (profiles/r05_s24: the wait per step 0.4-0.7 µs at depth 2,
        0.003 µs at 32); the shared-memory and host transports keep 2."""
        if self.lockstep_depth is not None:
            return self.lockstep_depth
        return 32 if transport == "rccl" and self.plan.device_decode else 2

    def _lockstep_commit_every(self, transport) -> int:
        """Tuning.lockstep_commit_every, or its auto value per transport: 4 on the shared-memory
        transport (an agreement costs well under a microsecond: 4.5 batches per commit, p99 commit
        latency 40 µs, no cost, profiles/r06_s5); 0 over RCCL and the host all-reduce, where each
        agreement costs the loader tens of microseconds (RCCL at world 1: commit_every=32 gives 32.5
        batches per commit and a p99 commit latency of 279 µs but costs 21 %; 0 gives ~220 and
        about 3 %, profiles/r06_s5, r05_s24)."""
        if self.lockstep_commit_every is not None:
            return self.lockstep_commit_every
        return 4 if transport == "shm" else 0

    def _single_host(self, process_group=None, probe: bool = False):
        """True when every rank of the group runs on this host.  From torchrun's environment
        (LOCAL_WORLD_SIZE == WORLD_SIZE) when it is there; else, with ``probe``, one all-gather of
        the ranks' host keys over a CPU group (a collective: only where every rank gets to);
        None when unknown."""
        import os

        import torch.distributed as dist

        world = dist.get_world_size(process_group)
        if world == 1:
            return True
        cache = self.__dict__.setdefault("_single_host_cache", {})
        key = None if process_group is None else tuple(dist.get_process_group_ranks(process_group))
        if key in cache:
            return cache[key]
        lws, ws = os.environ.get("LOCAL_WORLD_SIZE"), os.environ.get("WORLD_SIZE")
        if process_group is None and lws and ws and int(ws) == world:
            cache[key] = int(lws) == int(ws)
            return cache[key]
        if not probe:
            return None
        keys = [None] * world
        dist.all_gather_object(keys, _host_key(), group=self._gloo_of(process_group))
        cache[key] = len(set(keys)) == 1
        return cache[key]

    def _gloo_of(self, process_group):
        import torch.distributed as dist

        if dist.get_backend(process_group) == "gloo":
            return process_group
        cache = self.__dict__.setdefault("_lockstep_gloo", {})
        key = None if process_group is None else tuple(dist.get_process_group_ranks(process_group))
        if key not in cache:
            ranks = None if process_group is None else list(key)
            cache[key] = dist.new_group(ranks=ranks, backend="gloo")  # collective: every rank gets here
        return cache[key]

    def _lockstep_transport(self, process_group=None, probe: bool = False):
        """How ranks agree on every step: 'shm' (every rank on this host: the node-local shared-memory
        transport), 'rccl' (native communicator: an nccl process group across hosts, or
        lockstep='rccl'), 'host' (the process group's all-reduce), or None (no lockstep)."""
        # True: at world size > 1; "always" and a forced transport: at any world size (world 1
        # rehearses the per-step agreement on one GPU)
        if not self.lockstep or (self.lockstep is True and self.world_size <= 1):
            return None
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()):
            return None
        if self.lockstep in ("rccl", "host", "shm"):
            forced = self.lockstep
            if forced == "rccl" and (self.device.type != "cuda" or not self.native):
                forced = "host"
            return forced
        if self._single_host(process_group, probe):
            return "shm"
        if self.device.type != "cuda" or not self.native:
            return "host"
        return "rccl" if dist.get_backend(process_group) == "nccl" else "host"

    def _make_shm_lockstep(self, process_group, module):
        """The node-local transport (csrc/core/shm_lockstep.h): rank 0 makes the segment and names it
        over a CPU group, every rank maps it, then the name is removed (nothing stays in /dev/shm)."""
        import torch.distributed as dist

        rank = dist.get_rank(process_group)
        world = dist.get_world_size(process_group)
        grp = self._gloo_of(process_group)
        slots = max(8, self._lockstep_depth("shm") + 4)
        name = [module.ShmLockstep.create(world, slots) if rank == 0 else None]
        src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        dist.broadcast_object_list(name, src=src, group=grp, device=torch.device("cpu"))
        try:
            ls = module.ShmLockstep(name[0], rank, world)
        finally:
            dist.barrier(group=grp)  # every rank attached (or failed to) before the name goes
            if rank == 0:
                try:
                    os.unlink("/dev/shm/" + name[0].lstrip("/"))
                except FileNotFoundError:
                    pass
        ls.set_timeout_ms(int(self.lockstep_timeout * 1000))
        # start-up proof that the segment spans the whole group: one sum of the rank ids through it
        rank_sum = int(ls.allreduce_sum(rank))
        if int(ls.attached) != world or rank_sum != world * (world - 1) // 2:
            raise RuntimeError(f"lockstep: shared-memory segment has {ls.attached} ranks (rank-id sum {rank_sum}), "
                               f"the process group {world}: are the ranks on different hosts?")
        self.lockstep_info = {"transport": "shm", "world_size": world, "rank_id_sum": rank_sum, "slots": slots,
                              "what": "node-local shared-memory all-reduce(MIN) of the agreement words"}
        return ls

    def _make_rccl_lockstep(self, process_group):
        """Native RCCL communicator for the per-step lockstep (id broadcast through torch.distributed)."""
        import torch.distributed as dist

        lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        rank = dist.get_rank(process_group)
        world = dist.get_world_size(process_group)
        uid = [hip().RcclLockstep.unique_id(lib) if rank == 0 else None]
        src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        # the id travels over a CPU (gloo) group: broadcasting it over an nccl group would create
        # torch's own RCCL communicator -- and its streams, which take hardware queues -- for one
        # 128-byte message
        via_group = process_group
        if dist.get_backend(process_group) != "gloo":
            ranks = None if process_group is None else dist.get_process_group_ranks(process_group)
            via_group = dist.new_group(ranks=ranks, backend="gloo")  # collective: every rank gets here
        dist.broadcast_object_list(uid, src=src, group=via_group, device=torch.device("cpu"))
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        ls = hip().RcclLockstep(lib, uid[0], rank, world, dev, self._lockstep_depth("rccl") + 2)
        ls.set_timeout_ms(int(self.lockstep_timeout * 1000))
        # start-up proof that the communicator spans the whole job: RCCL's own count of its ranks,
        # and one all-reduce of the rank ids over it
        nranks = int(ls.nranks)
        rank_sum = int(ls.allreduce_sum(rank))
        if nranks != world or rank_sum != world * (world - 1) // 2:
            raise RuntimeError(f"lockstep: RCCL communicator has {nranks} ranks (rank-id sum {rank_sum}), "
                               f"the process group {world}")
        self.lockstep_info = {"transport": "rccl", "rccl_nranks": nranks, "rank_id_sum": rank_sum,
                              "world_size": world, "words": ls.words_mode,
                              "stream": ("greatest priority: a hardware-queue pool of its own" if ls.high_priority
                                         else "normal priority (shares the process's queues)")}
        return ls

    def _torch_nccl_active(self) -> bool:
        """torch makes its RCCL communicator (and streams) at a group's first collective: a DDP
        job's gradient all-reduce does at world > 1 (bench.py's world-1 rehearsal says so)."""
        try:
            import torch.distributed as dist

            return bool(dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"
                        and (dist.get_world_size() > 1 or os.environ.get("TORCHKAFKA_TORCH_NCCL_ACTIVE") == "1"))
        except Exception:  # noqa: BLE001
            return False

    def _decode_streams_fitting(self, copy_streams: int) -> int:
        """Decode streams that fit beside the other streams of the process in its hardware queues,
        when a collective shares the GPU with the loader (torch's NCCL stream, the RCCL lockstep);
        otherwise the engine's default (3: the loader's own streams may share a queue)."""
        try:
            rccl = self._lockstep_transport() == "rccl" and os.environ.get("TORCHKAFKA_LOCKSTEP_PRIORITY") != "high"
        except Exception:  # noqa: BLE001 - no process group to ask: no lockstep
            rccl = False
        nccl = self._torch_nccl_active()
        if not (rccl or nccl):
            return 3
        hw = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        reserved = 1 + int(nccl) + int(rccl) + copy_streams + (2 if self.plan.mirror else 0)  # mirror: 2 SDMA streams
        return max(1, min(3, hw - reserved))

    def stream_plan(self) -> dict:
        """The HIP streams the live iteration uses, against the process's hardware queues
        (``GPU_MAX_HW_QUEUES``, 4 by default).  HIP binds streams to queues round-robin in creation
        order, so past that count two streams share a queue and a launch on one can wait behind
        the other's (e.g. a decode kernel behind a collective waiting for the other ranks)."""
        run = self._run
        plan = {"user": 1, "decode": 0, "copy": 0, "mirror_copy": 0, "rccl_lockstep": 0, "torch_nccl": 0}
        if run is not None and run.engine is not None:
            plan["decode"] = int(run.engine.decode_streams()) if self.plan.device_decode else 0
            plan["copy"] = int(run.engine.copy_streams())
            if run.driver is not None:
                plan["mirror_copy"] = int(run.driver.mirror_copy_streams)
        if run is not None and run.rccl is not None and self.lockstep_info.get("transport") == "rccl":
            # a greatest-priority stream takes a queue from the high-priority pool, not these
            plan["rccl_lockstep"] = 0 if getattr(run.rccl, "high_priority", False) else 1
            plan["rccl_lockstep_high_priority"] = 1 - plan["rccl_lockstep"]
        # the lockstep never runs a collective on torch's group; a DDP job's gradient all-reduce does
        plan["torch_nccl"] = int(self._torch_nccl_active())
        total = sum(v for k, v in plan.items() if k != "rccl_lockstep_high_priority")
        hw = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        plan.update(total=total, hw_queues=hw, shared=total > hw)
        return plan
