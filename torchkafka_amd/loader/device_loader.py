"""DeviceLoader: Kafka records -> collated device tensors with exact per-batch commits.

Data path per batch (MI355X-first, no torch DataLoader on the hot path):

  worker process                         main process                       GPU
  ----------------------------------    ---------------------------------  -----------------------------
  fetch RecordBatches from the broker
  log, CRC-check, None-skip filter,
  pack values into a pinned ring slot
  (native C++; or `_process` + stack)
  publish slot (futex)          ----->  acquire READY slot
                                        hipMemcpyAsync slot -> staging      copy stream (side stream)
                                        (issued `prefetch` batches ahead,
                                         so the copy of k+1 overlaps the
                                         user's step k)
                                        stream-wait(h2d event)               compute stream:
                                        collate kernel launch        ----->  stack/pad + cast bf16/fp8
                                                                             (+ fused normalisation)
                                        slot FREE once its DMA is done
                                        yield device tensor
  ...                                   next(): commit batch k's offset
                                        watermarks to the broker (exact),
                                        lock-stepped over RCCL when DDP

Every slot carries the exact per-partition offsets of the records packed in
it, so commits cover exactly what the user has finished (reference D3),
whatever the prefetch depth and whichever worker produced the batch (D5).
"""
from __future__ import annotations

import ctypes
import gc
import logging
import multiprocessing as mp
import os
import threading
import time
import uuid
from collections import deque
from typing import NamedTuple

import torch

from ..client.errors import CorruptRecordException
from ..config import LoaderConfig
from ..ops.collate import CODE_DTYPE, DTYPE_CODE, FLOAT_DTYPES, _stream_ptr, normalize_params
from ..ops.native import core, hip
from ..parallel.sharding import dist_rank_world
from ..utils import topology
from ..utils.metrics import LoaderStats
from ..utils.tracing import enabled as _roctx_enabled
from ..utils.tracing import trace_range
from .bridging import LoaderBridges
from .commits import LoaderCommits
from .path_plan import PathPlan
from .worker import worker_main

log = logging.getLogger(__name__)
_ds_logger = logging.getLogger("torchkafka.kafka_dataset")


def _traced_step(step):
    """A native iteration step inside one roctx range (``TORCHKAFKA_ROCTX=1``)."""
    def traced():
        with trace_range("torchkafka.next_batch"):
            return step()
    return traced


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


class KafkaBatch(NamedTuple):
    """Batch plus provenance (``return_info=True``)."""

    data: torch.Tensor
    lengths: torch.Tensor | None
    mask: torch.Tensor | None
    watermarks: list      # [(pidx, first_offset, next_offset, n_records)]
    n_records: int        # records consumed incl. skipped ones


class WorkerError(RuntimeError):
    pass


class _PackerThread(threading.Thread):
    """num_workers=0: the ring producer as a thread of the main process (looks like a worker
    process to the liveness checks)."""

    def __init__(self, ring, name, dataset, cfg):
        super().__init__(target=worker_main, args=(ring, name, 0, 1, dataset, None, cfg), daemon=True,
                         name="torchkafka-packer")
        self.pid = os.getpid()

    @property
    def exitcode(self):
        return None if self.is_alive() else 0

    def terminate(self):  # stops at ring.shutdown(); nothing to signal
        pass


class _Run:
    """Resources of one iteration: ring, worker processes, H2D engine."""

    def __init__(self, loader: "DeviceLoader"):
        self.loader = loader
        L = loader
        self.name = f"/tkring-{os.getpid()}-{uuid.uuid4().hex[:10]}"
        self.ring = core().Ring.create(self.name, L.n_producers, L._slots_per_worker(), L._slot_capacity())
        self.procs: list = []
        self.engine = None
        self.driver = None
        self.rccl = None
        self.payload_addr = [self.ring.payload_address(g) for g in range(self.ring.n_slots)]
        self.staged: deque = deque()       # (g, summary, wms) with H2D issued (or CPU: just acquired)
        self.inflight: list = []           # slots whose H2D may still be reading host memory
        self.done = [False] * L.n_producers
        self.carry: list = []              # watermarks of consumed-but-undelivered records
        self.closed = False
        if L.numa_bind and L.device.type == "cuda" and L.device.index is not None:
            # before the fork: the workers inherit the mask, and the ring pages they first-touch land on
            # the GPU's socket (utils/topology.py)
            topology.bind_to_gpu_numa(L.device.index)
        ctx = mp.get_context(L.multiprocessing_context)
        cfg = L._worker_cfg()
        self.table = None          # commit_sink='worker': finished offsets published to the workers
        self.pidx_worker: dict = {}
        if L._sink == "worker":
            from .commit_channel import WatermarkTable

            self.table = WatermarkTable(L.n_producers)
            cfg["commit_table"] = self.table
        pass_ring = L.multiprocessing_context == "fork"
        try:
            if L.num_workers == 0:
                # single-process mode: the packer runs in a thread of this process (the native fill
                # releases the GIL), on the dataset's own consumer
                cfg["in_process"] = True
                t = _PackerThread(self.ring, self.name, L.dataset, cfg)
                t.start()
                self.procs.append(t)
            # A forked child must never run the finalizers of the parent's objects: when this process
            # already initialised HIP (a second epoch, a test session), a garbage CUDA tensor
            # collected in the child calls into a runtime that does not exist there (SIGSEGV right
            # after the fork, measured).  Collect now and freeze what is left out of the child's GC.
            frozen = pass_ring and L.num_workers > 0
            if frozen:
                gc.collect()
                gc.freeze()
            try:
                for w in range(L.num_workers):
                    p = ctx.Process(target=worker_main,
                                    args=(self.ring if pass_ring else None, self.name, w, L.num_workers,
                                          L.dataset, L.worker_init_fn, cfg),
                                    daemon=True, name=f"torchkafka-worker-{w}")
                    p.start()
                    self.procs.append(p)
            finally:
                if frozen:
                    gc.unfreeze()
            if L.device.type == "cuda":
                # only after the fork: workers never inherit an initialised HIP runtime state they would use
                dev = L.device.index if L.device.index is not None else torch.cuda.current_device()
                # device decode with h2d='dma': the slots (row tables) are read zero-copy and the copy
                # engines move the log bytes into an HBM mirror (enable_mirror below)
                mode = hip().H2D_ZERO_COPY if (L.plan.resolve_h2d(self.ring.payload_capacity) in ("zerocopy", "direct")
                                               or L.plan.mirror) else hip().H2D_DMA
                self.engine = hip().Engine(dev, self.ring.n_slots, self.ring.payload_capacity, L.copy_streams, mode)
                if L.tuning.decode_streams is not None:  # before anything creates a decode stream
                    self.engine.set_decode_streams(int(L.tuning.decode_streams))
                elif L._lockstep_transport() == "rccl":
                    # HIP gives a process 4 hardware queues: the user's stream, two decode streams and
                    # the lockstep's RCCL stream each keep one, so a collective waiting for the other
                    # ranks never sits in front of a decode kernel those ranks' progress depends on
                    self.engine.set_decode_streams(2)
                if L.numa_bind:
                    topology.check_device(dev)
                url, group = L._commit_target_url()
                self.driver = hip().MainDriver(self.engine, self.name, url, group, L.prefetch, L.in_order,
                                               L._default_src_code())
                self.driver.set_commit_on_device(L.commit_on == "device")
                if self.table is not None:
                    self.driver.set_worker_sink(self.table.address, L.n_producers, self.table.capacity)
                self.driver.set_event_every(L._event_every(self.ring.n_slots))
                self.driver.set_coalesce(L.coalesce)
                self.driver.set_coalesce_wait_us(L.coalesce_wait_us if L.coalesce > 1 else 0)
                if L.plan.direct:
                    self.driver.enable_direct()
                if L.plan.direct or L.plan.device_decode:
                    self.driver.pin_logs(L._rank_partitions())
                if L.plan.mirror:
                    # under the RCCL lockstep one SDMA copy stream: the process's 4 hardware queues
                    # go to the user's stream, two decode streams and the lockstep's RCCL stream
                    mcs = 1 if L._lockstep_transport() == "rccl" else 0
                    self.driver.enable_mirror(int(L.tuning.mirror_chunk_mib) << 20, int(L.tuning.mirror_chunks), mcs)
                tun = L.tuning
                if tun.ahead_depth is not None:
                    self.driver.set_ahead_depth(int(tun.ahead_depth))
                self.driver.set_group_bytes(int(tun.group_mib) << 20)
                # var-len / JSON device decode: the launches of the groups decoded ahead go through the
                # HIP command queue (csrc/hip/hip_queue.h; config 4 +9 %); fixed-width decode keeps
                # them on this thread (the 20-step headline lost 12 % to the queue's hand-off)
                self.driver.set_command_queue(bool(L.plan.json_span or L.plan.var_span))
        except BaseException:
            self.close()
            raise

    # ------------------------------------------------------------------ slot acquisition
    def _check_workers(self) -> None:
        for w, p in enumerate(self.procs):
            if not self.done[w] and not p.is_alive():
                raise WorkerError(f"DeviceLoader worker {w} (pid {p.pid}) exited unexpectedly "
                                  f"with exit code {p.exitcode}")

    def _check_workers_native(self) -> None:
        for w, p in enumerate(self.procs):
            if not p.is_alive() and not self.driver.worker_done(w):
                raise WorkerError(f"DeviceLoader worker {w} (pid {p.pid}) exited unexpectedly "
                                  f"with exit code {p.exitcode}")

    def acquire(self, block: bool):
        """Next READY slot as (g, summary, wms), or None (nothing ready / end of stream)."""
        ring = self.ring
        in_order = self.loader.in_order
        deadline = None if self.loader.timeout <= 0 else time.monotonic() + self.loader.timeout
        while True:
            g = ring.main_acquire(100 if block else 0, in_order)
            if g == -2:
                return None  # every worker delivered end-of-stream
            if g < 0:
                if not block:
                    return None
                self._check_workers()
                if deadline is not None and time.monotonic() > deadline:
                    raise TimeoutError(f"DeviceLoader timed out after {self.loader.timeout}s waiting for a batch")
                continue
            summ = ring.slot_summary(g)
            n_rows, flags = summ[0], summ[1]
            if flags & core().SLOT_ERROR:
                err = ring.slot_info(g)["error"]
                ring.main_release(g)
                raise WorkerError(err)
            if flags & core().SLOT_EOS:
                w = summ[6]
                self.done[w] = True
                ring.mark_done(w)
            wms = ring.watermarks(g)
            if self.table is not None:
                for w in wms:
                    self.pidx_worker[w[0]] = summ[6]
            if n_rows == 0:
                # empty (end-of-stream) slot: no data, but its watermarks may cover skipped records;
                # it stays in delivery order so they are committed after the worker's earlier batches
                ring.main_release(g)
                if not wms:
                    continue
                return g, summ, wms
            if self.engine is not None:
                self.engine.h2d(g, self.payload_addr[g], summ[2])
                self.inflight.append(g)
            return g, summ, wms

    def release_completed(self) -> None:
        if not self.inflight:
            return
        keep = []
        for g in self.inflight:
            if self.engine.h2d_complete(g):
                self.ring.main_release(g)
            else:
                keep.append(g)
        self.inflight = keep

    def wait_worker_commits(self, timeout: float) -> bool:
        """commit_sink='worker': waits until every live worker acknowledged its latest request."""
        return self.table.wait_acks(timeout=timeout, alive=lambda w: self.procs[w].is_alive()
                                    if w < len(self.procs) else False)

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        if self.table is not None:
            # the workers' consumers commit what the user finished before they are stopped
            self.wait_worker_commits(10.0)
        try:
            self.ring.shutdown()
        except Exception:  # noqa: BLE001
            pass
        for p in self.procs:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=5)
        if self.engine is not None:
            try:
                self.engine.synchronize()
            except Exception:  # noqa: BLE001
                log.exception("engine teardown failed")
        self.driver = None  # unregisters its pinned ring mapping
        self.rccl = None
        self.engine = None
        if self.table is not None:
            self.table.close()
        try:
            self.ring.unlink()
        except Exception:  # noqa: BLE001
            pass


class DeviceLoader(LoaderBridges, LoaderCommits):
    """Streams a :class:`KafkaDataset` to device tensors.

    Mirrors ``DataLoader(dataset, batch_size, num_workers, worker_init_fn)``
    (reference README.md:109-127) and adds the device path.  Iterate it
    directly (no commits; call :meth:`commit`) or through
    :func:`~torchkafka_amd.auto_commit` (commit after every batch).

    Args:
        dataset: a ``KafkaDataset`` placeholder (workers build consumers via ``worker_init_fn``), or
            -- with ``num_workers=0`` -- a dataset built with its consumer (``YourDataset(topic, ...)``).
        batch_size: records per batch (per rank).
        num_workers: consumer/packer processes; 0 = the reference's single-process mode
            (auto_commit.py:49-58): a thread of this process consumes and packs the pinned ring
            slots with the dataset's own consumer, and the device path is unchanged.
        worker_init_fn: usually ``YourDataset.init_worker(topic, group_id=..., bootstrap_servers=...)``.
        device: target device (default: current CUDA device, else CPU).
        dtype: output dtype (default: the schema's); floats may go to bf16/f16/fp8 (OCP e4m3fn).
        config: a :class:`~torchkafka_amd.config.LoaderConfig` (or its dict form).  Every field below
            can also be passed as a keyword argument, which overrides the config; the performance
            knobs (``slots_per_worker``, ``slot_bytes``, ``prefetch``, ``copy_streams``,
            ``event_every``, ``coalesce``, ``coalesce_wait_us``, ``lockstep_depth``, ``numa_bind``,
            ``ahead_depth``, ``decode_streams``, ``worker_spin_us``, ``json_count``, ...) form its
            :class:`~torchkafka_amd.config.Tuning` (docs/CONFIG.md).  Options:
        normalize: optional ``(mean, std)`` fused into the collate kernel.
        sharding: ``"static"`` rank/worker partition map (default) or ``"group"`` (Kafka group assignment).
        slots_per_worker: ring depth per worker (prefetched batches in pinned memory).  Default: as
            deep as 8 slots while the whole ring stays within 64 MiB of pinned memory (at least 4).
            Slots whose kernels are still queued on the GPU stay held, so a shallow ring starves
            the workers (config 2 on MI355X: 4 slots 29-31 M rec/s, 8 slots 30-33 M).
        prefetch: batches whose H2D copy is issued ahead of the user (overlap with compute).
        in_order: strict worker round-robin (reference order) instead of first-ready.
        pad_to: var-len / JSON batches are padded to this fixed width (use the schema's ``max_len`` /
            ``truncate`` to bound the rows); None pads each batch to its longest row.
        pad_multiple: with ``pad_to=None``, the batch width is rounded up to a multiple of this.
        pad_value: the value written into the padding.
        return_mask: var-len / JSON batches also yield a bool ``[rows, width]`` mask of real elements.
        drop_last: drop a final batch shorter than ``batch_size`` (DataLoader's meaning).
        return_info: yield ``(batch, BatchInfo)`` with each batch's partitions and offset ranges.
        native: use the native step driver (``False``: the Python loop, for debugging).
        multiprocessing_context: start method of the worker processes (``"fork"``, ``"spawn"``,
            ``"forkserver"``).
        commit_sink: ``"broker"`` (this process stores finished offsets into the synthetic broker),
            ``"worker"`` (each worker's consumer commits its own partitions, as the reference) or
            ``"auto"`` (broker when the workers read the synthetic broker with static sharding).
        rank: this process's rank for static sharding (default: torch.distributed's, else 0).
        world_size: ranks sharing the topic (default: torch.distributed's, else 1).
        timeout: seconds to wait for a batch before ``TimeoutError`` (0 waits forever).
        group_id: consumer group the commits go to (default: the one given to ``init_worker``).
        bootstrap_servers: where the group lives (default: the one given to ``init_worker``).
        base_seed: seed of the workers' RNGs (worker k gets ``base_seed + k``); None draws one from torch.
        decode: ``"device"`` (fixed-width / var-len records decoded by the gfx950 kernels straight from
            the pinned broker logs, CRC32C included; the workers only walk record headers),
            ``"host"`` (the workers CRC-check and pack the values) or ``"auto"`` (device when possible).
        json_parse: ``JsonArray`` records parsed by the gfx950 kernel (``"device"``), by the workers
            (``"host"``), or ``"auto"`` (device unless ``skip_bad=True`` needs rows dropped).
        bridge: ``"auto"``: workers pointed at a real Kafka cluster read a local replica that a native
            ``KafkaBridge`` fills with this rank's partitions (commits reach the cluster's coordinator);
            ``True`` requires it, ``False`` lets the workers' consumers read the cluster themselves.
        commit_on: ``"host"`` (commit when the next batch is requested, as the reference) or
            ``"device"`` (additionally wait until the GPU finished the user's work on the batch).
        commit: ``"async"`` (default: batch k's offsets are stored -- in the synthetic broker, or in a
            KafkaBridge replica that forwards them to the group coordinator within a few ms -- when
            batch k+1 is requested) or ``"sync"`` (the reference's semantics, kafka_dataset.py:130:
            batch k+1 is handed out only after batch k's device verdict landed, its offsets were
            stored and, through a bridge, the coordinator answered its OffsetCommit).  Under a
            cross-rank lockstep the same holds on every rank: before batch k+1 is taken, one
            agreement issued at step k+1 proves every rank finished batch k, and each rank commits
            its own part of batch k before it hands out k+1 (one collective per step).
        verify: ``"deliver"`` (a batch decoded or parsed on the GPU is handed out only once its
            kernel's verdict -- every RecordBatch's CRC32C, every JSON row's grammar -- landed; a
            corrupt batch raises ``CorruptRecordException`` before it is yielded, as kafka-python's
            ``check_crcs`` iterator raises before ``_process`` sees a record) or ``"commit"`` (the
            verdict gates only the commit: the batch may be yielded while its kernel still runs and
            the exception comes one or more steps later).  Host-decoded batches are verified by the
            workers before they are published, in both modes.
        lockstep: synchronise steps and commits across ranks when torch.distributed is initialised
            (``True``: native RCCL on GPUs with an nccl group, the group's own all-reduce otherwise;
            ``"host"``: the group's all-reduce (e.g. gloo) even on GPUs; ``"rccl"``: the native RCCL
            transport whatever the group's backend; ``"always"``: also at world size 1).
        lockstep_depth: steps the per-step agreement is issued ahead (hides the collective's latency).
        h2d: ``"dma"`` (hipMemcpyAsync into device staging on ``copy_streams`` side streams, issued
            ``prefetch`` batches ahead), ``"zerocopy"`` (the collate kernel reads pinned host memory over
            PCIe: two HIP calls per batch instead of five, but the read runs on the compute stream) or
            ``"auto"`` (default: zero-copy for slots up to ``ZERO_COPY_MAX_BYTES``, where a batch is
            latency-bound; DMA above, where copy/compute overlap matters; var-len / JSON rows decoded
            on the device read an HBM mirror of the logs that the copy engines fill, fixed-width rows
            read the pinned logs in place -- loader/path_plan.py) or ``"direct"`` (experimental;
            fixed-width schemas on the synthetic broker: workers only locate each row in the broker log,
            the main process pins the logs in place and the collate kernel gathers rows straight out of
            them over PCIe, so no worker copies the payload.  Measured slower than "zerocopy" on MI355X
            (docs/PERFORMANCE.md): the CPU CRC pass still dominates a worker, the gather kernel pays a
            second dependent PCIe round trip, and pinning new log pages runs at ~13 GB/s).
        event_every: record a slot-completion event for one batch in k (default: ring slots / 4,
            at most 4); slots in between are released with the next event on the same stream.
        coalesce: fixed-width batches that are already staged when the next one is requested are
            collated together, up to this many per kernel launch (one allocation, one launch, one
            completion event); the following requests return them without a HIP call.  1 disables.
        coalesce_wait_us: while the GPU is still busy with an earlier launch, wait up to this long
            for enough staged batches to fill a group (costs no GPU time; a zero-copy batch takes
            7.1 us alone and 5.2 us in a group of 4).  0 launches whatever is staged at once.
        lockstep_timeout: seconds the native RCCL lockstep waits for the other ranks before it
            aborts its communicator and raises (a peer died or hung); <= 0 waits forever.
        numa_bind: before forking the workers, restrict this process (and so the workers) to the CPUs
            of the socket the target GPU is attached to (no-op on single-socket hosts or when
            ``TORCHKAFKA_NUMA=0``); see ``utils/topology.py``.
    """

    def __init__(self, dataset, batch_size: int = 256, *, num_workers: int = 4, worker_init_fn=None,
                 device=None, dtype: torch.dtype | None = None, config: LoaderConfig | dict | None = None,
                 **options):
        if batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        if num_workers < 0:
            raise ValueError("num_workers must be >= 0")
        cfg = self.config = LoaderConfig.build(config, **options)
        tun = cfg.tuning
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.num_workers = int(num_workers)
        self.worker_init_fn = worker_init_fn
        if self.num_workers == 0:
            # the reference's single-process mode (auto_commit.py:49-58): the dataset was built with
            # its consumer in this process; a thread of this process packs the ring slots
            if getattr(dataset, "_consumer", None) is None:
                raise ValueError("DeviceLoader(num_workers=0) needs a dataset with its consumer, e.g. "
                                 "YourDataset('topic', bootstrap_servers=..., group_id=...), not a placeholder")
            if worker_init_fn is not None:
                raise ValueError("worker_init_fn is not used with num_workers=0 (there are no workers)")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.schema = getattr(dataset, "schema", None)
        self.dtype = dtype
        # behaviour (config.LoaderConfig)
        self.normalize = cfg.normalize
        self.sharding = cfg.sharding
        self.in_order = cfg.in_order
        self.drop_last = cfg.drop_last
        self.pad_to = cfg.pad_to
        self.pad_multiple = int(cfg.pad_multiple)
        self.pad_value = cfg.pad_value
        self.return_mask = cfg.return_mask
        self.return_info = cfg.return_info
        self.native = cfg.native
        self.multiprocessing_context = cfg.multiprocessing_context
        self.commit_on = cfg.commit_on
        self.commit_mode = cfg.commit
        self.verify = cfg.verify
        self.commit_sink = cfg.commit_sink
        self.lockstep = cfg.lockstep
        self.lockstep_timeout = float(cfg.lockstep_timeout)
        self.lockstep_info: dict = {}  # how the last iteration agreed across ranks (bench / logs)
        self.h2d = cfg.h2d
        self.json_parse = cfg.json_parse
        self.decode = cfg.decode
        self.timeout = cfg.timeout
        r, w = dist_rank_world()
        self.rank = r if cfg.rank is None else int(cfg.rank)
        self.world_size = w if cfg.world_size is None else int(cfg.world_size)
        self.base_seed = (int(torch.empty((), dtype=torch.int64).random_().item()) if cfg.base_seed is None
                          else cfg.base_seed)
        # performance (config.Tuning)
        self.tuning = tun
        self.slots_per_worker = None if tun.slots_per_worker is None else int(tun.slots_per_worker)
        self.slot_bytes = tun.slot_bytes
        self.prefetch = int(tun.prefetch)
        self.copy_streams = int(tun.copy_streams)
        self.event_every = None if tun.event_every is None else int(tun.event_every)
        self.coalesce = int(tun.coalesce)
        self.coalesce_wait_us = int(tun.coalesce_wait_us)
        self.lockstep_depth = None if tun.lockstep_depth is None else int(tun.lockstep_depth)
        self.numa_bind = bool(tun.numa_bind)
        self._bridges: list = []
        if self.num_workers > 0 and cfg.bridge is not False:
            self.worker_init_fn = self._bridge_cluster(self.worker_init_fn, forced=cfg.bridge is True)
        self._group_id, self._servers = self._resolve_commit_target(cfg.group_id, cfg.bootstrap_servers)
        self._sink = self._resolve_sink()
        self.plan = PathPlan.build(
            device_type=self.device.type, schema=self.schema, native=self.native, decode=self.decode, h2d=self.h2d,
            json_parse=self.json_parse, synthetic_commits=self._commit_target_url()[0] != "",
            process_overridden=self._process_overridden(), return_info=self.return_info,
            drop_last=self.drop_last, json_count_mode=getattr(tun, "json_count", "auto"))
        self._pending_wms: list = []   # finished-but-uncommitted watermark lists
        self._committed: dict[int, int] = {}
        # state_dict(global_step=True): every partition's position after the batches handed out
        # (this loader's lifetime, and the checkpoint it resumed from) and how many steps that is
        self._delivered_pos: dict[int, int] = {}
        self._steps_delivered = 0
        self._global_step_base = 0
        self._norm = None
        self.stats = LoaderStats()
        self._run: _Run | None = None

    @property
    def n_producers(self) -> int:
        """Ring producers: the worker processes, or the in-process packer thread (num_workers=0)."""
        return max(1, self.num_workers)

    # ------------------------------------------------------------------ configuration helpers

    def _resolve_sink(self) -> str:
        """Where finished offsets are committed.  'broker': this process stores them straight into
        the synthetic broker's offset table (one native store per batch) -- only valid when the
        workers are simple (manually assigned) consumers of a synthetic broker.  'worker': each
        worker's own consumer commits them: required with sharding='group' (a member's commit is
        tied to its generation) and with any other consumer (kafka-python)."""
        synthetic = self._commit_target_url()[0] != ""
        if self.commit_sink == "broker":
            if not synthetic or self.sharding != "static":
                raise ValueError("commit_sink='broker' needs the synthetic broker, a group_id and sharding='static'")
            return "broker"
        if self.commit_sink == "worker" or self.sharding == "group" or not synthetic:
            return "worker"
        return "broker"

    def _process_overridden(self) -> bool:
        """The dataset maps records with a ``_process`` of its own (reference kafka_dataset.py:159):
        the native schema packers and the device decode would bypass it, so the workers run the
        per-record loop and the batches take the generic path."""
        from ..models.kafka_dataset import KafkaDataset

        return type(self.dataset)._process is not KafkaDataset._process

    def _event_every(self, n_slots: int) -> int:
        """Slots per completion event: one ``hipEventRecord`` per batch costs ~1.3 µs of host time,
        so with a deep ring only every k-th batch records one (k <= n_slots / 4 keeps workers fed;
        measured on MI355X, config 2: k=1 21.5M, k=2 24.8M, k=4 29.1M records/s)."""
        if self.event_every is not None:
            return self.event_every
        return max(1, min(4, n_slots // 4))

    def _default_src_code(self) -> int:
        s = self.schema
        if s is None:
            return -1
        if getattr(s, "kind", None) == 2:
            return DTYPE_CODE[torch.float32]
        return DTYPE_CODE[s.dtype]

    def _slots_per_worker(self) -> int:
        if self.slots_per_worker is not None:
            return self.slots_per_worker
        try:
            rccl = self._lockstep_transport() == "rccl"
        except Exception:  # noqa: BLE001 - no process group to ask: no lockstep
            rccl = False
        return self.plan.slots_per_worker(self._slot_capacity(), self.n_producers, deep=rccl)

    def _lockstep_depth(self, transport) -> int:
        """Tuning.lockstep_depth, or its auto value: an RCCL agreement takes ~60-180 µs to come back
        while device-decoded steps take ~5 µs, so with the 64-deep ring the next one is issued 32
        steps before the credits run out (profiles/r05_s24: the wait per step 0.4-0.7 µs at depth 2,
        0.003 µs at 32); the host lockstep keeps 2."""
        if self.lockstep_depth is not None:
            return self.lockstep_depth
        return 32 if transport == "rccl" and self.plan.device_decode else 2

    def _n_extras(self) -> int:
        """Record-field columns (Key / Timestamp) the schema adds beside the value."""
        return len(getattr(self.schema, "fields", ()) or ())

    def _slot_capacity(self) -> int:
        if self.slot_bytes is not None:
            return int(self.slot_bytes)
        # record fields ride after the layout: one int64 per row each (+ alignment)
        nx = self._n_extras()
        return self.plan.layout_capacity(self.batch_size, self.schema) + (self.batch_size * 8 * nx + 256 if nx else 0)

    def _worker_cfg(self) -> dict:
        return {"batch_size": self.batch_size, "sharding": self.sharding, "rank": self.rank,
                "world_size": self.world_size, "native": self.native, "base_seed": self.base_seed,
                "gather": self.plan.direct, "json_device": self.plan.json_device, "json_count": self.plan.json_count,
                "span": self.plan.device_decode,
                "process_overridden": self.plan.process_overridden, "commit_table": None,
                "worker_spin_us": int(self.tuning.worker_spin_us), "in_process": False,
                "commit_mode": self.commit_mode}

    def _rank_partitions(self) -> list[int]:
        """Broker partition indices this rank's workers will read (static sharding of the topics
        given to ``init_worker``); empty when not known up front (group sharding, custom init)."""
        from ..models.kafka_dataset import _WorkerInit
        from ..parallel.sharding import shard_partitions

        wi = self.worker_init_fn
        if self.num_workers == 0:
            cons = getattr(self.dataset, "_consumer", None)
            topics = sorted(cons.subscription() or []) if cons is not None and hasattr(cons, "subscription") else []
        else:
            topics = list(wi.args) if isinstance(wi, _WorkerInit) else []
        if self.sharding != "static" or not topics:
            return []
        try:
            b = self._broker()
            out = []
            for topic in topics:
                if isinstance(topic, str) and b.has_topic(topic):
                    _, n, first = b.topic(topic)
                    out += [first + p for p in shard_partitions(n, self.rank, self.world_size)]
            return out
        except Exception:  # noqa: BLE001 - not a synthetic broker: pinned lazily, batch by batch
            return []

    def _out_dtype(self, src: torch.dtype) -> torch.dtype:
        if self.dtype is not None:
            return self.dtype
        return src

    def __len__(self):
        raise TypeError("a Kafka stream has no length")

    # ------------------------------------------------------------------ iteration
    def __iter__(self):
        return self._iterate(auto_commit=False)

    def _iterate(self, auto_commit: bool, process_group=None):
        if self._run is not None and not self._run.closed:
            raise RuntimeError("DeviceLoader is already being iterated")
        # fork the workers first: the lockstep below initialises HIP in this process
        run = self._run = _Run(self)
        lock = None
        try:
            transport = self._lockstep_transport(process_group)
            if transport is not None:
                import torch.distributed as dist

                if dist.is_available() and dist.is_initialized():
                    if run.driver is not None:
                        if transport == "rccl":
                            run.rccl = self._make_rccl_lockstep(process_group)
                        else:
                            run.rccl = hip().PyLockstep(_host_allreduce_min(process_group))
                            self.lockstep_info = {"transport": "host", "backend": dist.get_backend(process_group),
                                                  "world_size": dist.get_world_size(process_group)}
                        run.driver.enable_lockstep(run.rccl, self._lockstep_depth(transport))
                    else:
                        from ..parallel.lockstep import Lockstep

                        lock = Lockstep(process_group, None)
                        self.lockstep_info = {"transport": "host", "backend": dist.get_backend(process_group),
                                              "world_size": lock.world_size}
        except BaseException:
            run.close()
            raise
        if run.driver is not None:
            plan = self.stream_plan()
            if self.lockstep_info:
                self.lockstep_info["streams"] = plan
            if plan["shared"]:
                # measured: the lockstep on a shared normal-priority queue came back in ~60 µs, on a
                # queue of its own at the greatest priority in ~110 µs (profiles/r05_s19_rccl_matrix)
                log.debug("DeviceLoader: %d HIP streams on %d hardware queues (%s): some share a queue",
                          plan["total"], plan["hw_queues"], plan)
            yield from self._iterate_native(run, auto_commit)
            return
        finished = self._pending_wms
        prev = None
        step = 0
        completed = False
        try:
            sync = auto_commit and self.commit_mode == "sync"
            while True:
                item = self._next_item(run)
                status, fatal = 2, None
                if prev is not None and auto_commit:
                    finished.append(self._finish_marker(prev))  # the user is done with the previous batch
                    prev = None
                    if sync:
                        # commit='sync': batch k committed (and answered) BEFORE the agreement that
                        # hands out k+1, which carries how it went to every rank
                        try:
                            status = self._sync_commit_py()
                        except Exception as e:  # noqa: BLE001 - re-raised after the agreement
                            fatal, status = e, 0
                if lock is not None:
                    t_agree = time.perf_counter_ns()
                    try:
                        ok = lock.agree(item is not None, step, status)
                    except Exception as e:
                        if fatal is not None:
                            raise fatal from e
                        raise
                    t_agree = time.perf_counter_ns() - t_agree
                    st = self.stats
                    st.lockstep_agreements += 1
                    st.lockstep_wait_ns += t_agree
                    st.lockstep_step_wait_max_ns = max(st.lockstep_step_wait_max_ns, t_agree)
                    if auto_commit and not sync:
                        self._commit_finished()
                    if not ok:
                        break
                else:
                    if fatal is not None:
                        raise fatal
                    if auto_commit:
                        self._commit_finished()
                    if item is None:
                        break
                batch, wms = item
                if auto_commit:
                    prev = wms
                else:
                    finished.append((wms, None))  # manual mode: commit() covers every yielded batch
                pos = self._delivered_pos
                for pidx, _first, nxt, _n in wms:
                    if nxt > pos.get(pidx, -1):
                        pos[pidx] = nxt
                self._steps_delivered += 1
                step += 1
                yield batch
            completed = True
        finally:
            if completed and auto_commit:
                if prev is not None:
                    finished.append(self._finish_marker(prev))
                if run.carry:
                    finished.append((run.carry, None))
                    run.carry = []
                if lock is not None:
                    lock.barrier()
                self._commit_finished(wait=True)
                if self.commit_mode == "sync":
                    self._sync_commit_py()
            run.close()

    def _lockstep_transport(self, process_group=None):
        """How ranks agree on every step: 'rccl' (native communicator, an nccl process group or
        lockstep='rccl'), 'host' (the process group's all-reduce), or None (no lockstep)."""
        if not (self.lockstep and (self.world_size > 1 or self.lockstep == "always")):
            return None
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()):
            return None
        if self.device.type != "cuda" or not self.native:
            return "host"
        backend = dist.get_backend(process_group)
        return "rccl" if self.lockstep == "rccl" or (backend == "nccl" and self.lockstep != "host") else "host"

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
        try:
            import torch.distributed as dist

            # torch makes its RCCL communicator (and streams) at a group's first collective: the
            # lockstep never runs one on it, a DDP job's gradient all-reduce does (world > 1, or a
            # world-1 group that ran one: bench.py's rehearsal of the N = 8 queue layout)
            if (dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"
                    and (dist.get_world_size() > 1 or os.environ.get("TORCHKAFKA_TORCH_NCCL_ACTIVE") == "1")):
                plan["torch_nccl"] = 1
        except Exception:  # noqa: BLE001
            pass
        total = sum(v for k, v in plan.items() if k != "rccl_lockstep_high_priority")
        hw = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        plan.update(total=total, hw_queues=hw, shared=total > hw)
        return plan

    # ------------------------------------------------------------------ native iteration
    def _iterate_native(self, run: _Run, auto_commit: bool):
        """GPU iteration through the native step driver: one loop for every schema.  A *stage*
        makes one batch per call -- ``(status, commit status, item)`` -- and the loop around it
        owns what they share: result codes, commit logging, ``commit='sync'``, the wait timeout and
        the end of the iteration (final commit, stats, ring teardown).  Stages:

        * fixed-width (``FixedWidth`` schemas): ONE argument-free native call per batch (finish +
          commit the previous batch, take the next slot, allocate on the current stream, decode --
          coalesced with staged batches);
        * var-len / JSON (``VarLen`` / ``JsonArray``): the same with the pad/stack or JSON parse;
        * slot (everything else: ``return_info``, ``drop_last``, a ``_process`` of its own): the
          driver hands out slots and Python collates them.
        """
        drv = run.driver
        debug = _ds_logger.isEnabledFor(logging.DEBUG)
        log_commits = debug and auto_commit
        native_ac = auto_commit and not log_commits  # with DEBUG the commit comes back to Python to be logged
        if self.plan.fast_path:
            step, py_commits = self._fixed_stage(drv, native_ac), False
        elif self.plan.varlen_fast:
            step, py_commits = self._varlen_stage(drv, native_ac), False
        else:
            step, py_commits = self._slot_stage(run, auto_commit, debug), True
        if _roctx_enabled():
            step = _traced_step(step)
        sync = auto_commit and self.commit_mode == "sync"
        drv.set_sync_commit(sync)
        verify = self.verify == "deliver"
        completed = delivered = False
        wait_since = None
        try:
            while True:
                fatal = None
                if sync and delivered:
                    # commit='sync': asking for batch k+1 finishes batch k -- its verdict, its store
                    # and the coordinator's answer come FIRST, then the lockstep agreement that
                    # hands out k+1 carries how that went, so no rank sees k+1 before every rank
                    # committed k (the reference's auto_commit.py:55-58 / kafka_dataset.py:130 as a
                    # cross-rank barrier)
                    drv.finish_delivered(_stream_ptr(self.device))
                    try:
                        status = self._sync_commit(drv, debug)
                    except Exception as e:  # noqa: BLE001 - re-raised after the agreement
                        fatal, status = e, 0
                    drv.set_commit_status(status)
                    if fatal is not None and not drv.lockstep_enabled:
                        raise fatal
                try:
                    r, cs, item = step()
                except Exception as e:
                    if fatal is not None:
                        raise fatal from e
                    raise
                if cs:
                    self._log_commit(cs, debug)
                if r > 0 and verify and py_commits and drv.verify_delivered() < 0:
                    r = -5  # the fast stages wait for the verdict natively and return -5 themselves
                if r == -5:
                    # the batch's CRC32C / grammar verdict is bad: it never reaches the user (the
                    # reference's records pass kafka-python's check_crcs before _process sees them,
                    # kafka_dataset.py:156-162); the batches finished before it are committed first
                    if auto_commit and delivered:
                        self._commit_native(drv, debug)
                    raise CorruptRecordException(drv.parse_error())
                if r > 0:
                    if delivered and log_commits and not py_commits and not sync:
                        self._commit_logged(drv)
                    delivered = True
                    wait_since = None
                    self._steps_delivered += 1
                    yield item
                elif r == -2:
                    break
                elif r == -3:
                    raise WorkerError(drv.error())
                elif r == -4:  # an earlier device-checked batch was corrupt (manual-commit mode)
                    raise CorruptRecordException(drv.parse_error())
                else:  # -1: nothing within the poll slice
                    run._check_workers_native()
                    if self.timeout > 0:
                        now = time.monotonic()
                        wait_since = now if wait_since is None else wait_since
                        if now - wait_since > self.timeout:
                            raise TimeoutError(f"DeviceLoader timed out after {self.timeout}s waiting for a batch")
            completed = True
        finally:
            try:
                drv.finish_delivered(_stream_ptr(self.device))
                if completed:
                    drv.finish_lockstep()
                drv.drain_fenced(True)
                if completed and auto_commit:
                    self._commit_native(drv, debug)
                    if sync:
                        self._sync_commit(drv, debug)
                elif not auto_commit:
                    # manual mode: keep every yielded batch committable by DeviceLoader.commit()
                    pend = drv.take_pending()
                    if pend:
                        self._pending_wms.append(([(p, 0, o, 0) for p, o in pend], None))
            finally:
                self._absorb_driver_stats(drv)
                self._absorb_delivered(drv)
                run.close()

    def _fixed_stage(self, drv, native_ac: bool):
        s = self.schema
        prm = self._norm_params(s.row_elems)
        shift, scale = (prm[0].data_ptr(), prm[1].data_ptr()) if prm is not None else (0, 0)
        nx = self._n_extras()
        drv.configure_fast(self.device.index, [self.batch_size, *s.shape], DTYPE_CODE[self._out_dtype(s.dtype)],
                           s.row_elems, shift, scale, native_ac, 100, self.coalesce > 1, nx,
                           self.verify == "deliver")
        if nx < 2 or s.column_order() == list(range(nx)):
            return drv.fast_next
        order = s.column_order()  # fields added timestamp first: the native columns are key-first
        native = drv.fast_next

        def step():
            r, cs, item = native()
            if item is not None:
                item = (item[0], *(item[1 + i] for i in order))
            return r, cs, item
        return step

    def _varlen_stage(self, drv, native_ac: bool):
        src = CODE_DTYPE[self._default_src_code()]
        dst_dt = self._out_dtype(src)
        if (dst_dt in FLOAT_DTYPES) != (src in FLOAT_DTYPES) and src in FLOAT_DTYPES:
            raise TypeError(f"cannot collate {src} records to {dst_dt}")
        drv.configure_varlen(self.device.index, DTYPE_CODE[dst_dt], -1 if self.pad_to is None else int(self.pad_to),
                             self.pad_multiple, float(self.pad_value), bool(self.return_mask), native_ac, 100,
                             self.verify == "deliver")
        return drv.varlen_fast_next

    def _slot_stage(self, run: _Run, auto_commit: bool, debug: bool):
        drv = run.driver
        state = {"delivered": False}

        def step():
            drv.finish_delivered(_stream_ptr(self.device))  # asking for the next batch finishes the previous one
            if auto_commit and state["delivered"]:
                self._commit_native(drv, debug)
            item = self._next_item_driver(run)
            if item is None:
                return -2, 0, None
            drv.deliver_last()
            state["delivered"] = True
            return 1, 0, item[0]
        return step

    def _next_item(self, run: _Run):
        """Returns (batch, watermarks) or None at end of stream."""
        if run.driver is not None:
            return self._next_item_driver(run)
        t0 = time.perf_counter_ns()
        if run.engine is not None:
            run.release_completed()
        # top up the device-side prefetch (H2D of upcoming batches overlaps the user's step)
        while len(run.staged) < self.prefetch + 1:
            got = run.acquire(block=False)
            if got is None:
                break
            run.staged.append(got)
        if not run.staged:
            got = run.acquire(block=True)
            if got is None:
                return None
            run.staged.append(got)
        g, summ, wms = run.staged.popleft()
        t1 = time.perf_counter_ns()
        n_rows = summ[0]
        if n_rows == 0 or (self.drop_last and n_rows < self.batch_size):
            # nothing to deliver: carry the consumed offsets into the next delivered batch
            if n_rows and run.engine is None:
                run.ring.main_release(g)
            run.carry.extend(wms)
            return self._next_item(run)
        batch = self._collate(run, g, summ, wms)
        if run.carry:
            wms = run.carry + wms
            run.carry = []
        self.stats.record_batch(n_rows, summ[2], t1 - t0, time.perf_counter_ns() - t1)
        return batch, wms

    def _next_item_driver(self, run: _Run):
        drv = run.driver
        t0 = time.perf_counter_ns()
        while True:
            res = drv.next_slot(100)
            r = res[0]
            if r == -2:
                return None
            if r == -3:
                raise WorkerError(drv.error())
            if r == -4:
                raise CorruptRecordException(drv.parse_error())
            if r == -1:
                run._check_workers_native()
                if self.timeout > 0 and time.perf_counter_ns() - t0 > self.timeout * 1e9:
                    raise TimeoutError(f"DeviceLoader timed out after {self.timeout}s waiting for a batch")
                continue
            _, n_rows, kind, max_len, total, src_code, shape, payload_bytes = res
            wms = drv.last_watermarks()
            if self.drop_last and n_rows < self.batch_size:
                drv.discard_last()     # consumed but not handed out: finished right away
                drv.deliver_last()
                drv.finish_delivered()
                continue
            break
        t1 = time.perf_counter_ns()
        if kind == core().PACK_TREE:  # structured samples: one copy of the slot, leaves are views
            out = self._collate_tree(run, drv.last_slot, payload_bytes,
                                     lambda block: drv.copy_payload_last(_stream_ptr(self.device), block.data_ptr()))
            self.stats.record_batch(n_rows, payload_bytes, t1 - t0, time.perf_counter_ns() - t1)
            if self.return_info:
                return KafkaBatch(out, None, None, wms, sum(w[3] for w in wms)), wms
            return out, wms
        src_dt = CODE_DTYPE[src_code]
        dst_dt = self._out_dtype(src_dt)
        if (dst_dt in FLOAT_DTYPES) != (src_dt in FLOAT_DTYPES) and src_dt in FLOAT_DTYPES:
            raise TypeError(f"cannot collate {src_dt} records to {dst_dt}")
        dev = self.device
        stream = _stream_ptr(dev)
        lengths = mask = None
        # device-decode and log-gather slots are fixed-width batches too (MainDriver.collate_fixed)
        fixed = kind in (core().PACK_FIXED, core().PACK_RECORD_SPAN, core().PACK_GATHER_FIXED)
        if fixed:
            if not shape:
                shape = tuple(self.schema.shape)
            row = int(max_len) if max_len else 1
            out = torch.empty((n_rows, *shape), dtype=dst_dt, device=dev)
            prm = self._norm_params(row)
            shift, scale = (prm[0].data_ptr(), prm[1].data_ptr()) if prm is not None else (0, 0)
            nx = drv.last_extras
            ext = torch.empty((nx, n_rows), dtype=torch.int64, device=dev) if nx else None
            drv.collate_fixed_last(stream, DTYPE_CODE[dst_dt], out.data_ptr(), row, shift, scale,
                                   ext.data_ptr() if ext is not None else 0)
            if ext is not None and not self.return_info:
                out = self._with_fields(out, ext)
        else:
            L = self.pad_to if self.pad_to is not None else int(max_len)
            if self.pad_to is None and self.pad_multiple > 1:
                L = (L + self.pad_multiple - 1) // self.pad_multiple * self.pad_multiple
            out = torch.empty((n_rows, L), dtype=dst_dt, device=dev)
            lengths = torch.empty(n_rows, dtype=torch.int64, device=dev)
            mask = torch.empty((n_rows, L), dtype=torch.bool, device=dev) if self.return_mask else None
            W = drv.collate_varlen_last(stream, DTYPE_CODE[dst_dt], out.data_ptr(), L, float(self.pad_value),
                                        lengths.data_ptr(), mask.data_ptr() if mask is not None else 0,
                                        0 if self.pad_to is not None else max(1, self.pad_multiple))
            if W != L:  # device-counted JSON: L was the workers' bound, W the width the kernel chose
                out = out.view(-1)[:n_rows * W].view(n_rows, W)
                if mask is not None:
                    mask = mask.view(-1)[:n_rows * W].view(n_rows, W)
        self.stats.record_batch(n_rows, payload_bytes, t1 - t0, time.perf_counter_ns() - t1)
        n_rec = sum(w[3] for w in wms)
        if self.return_info:
            return KafkaBatch(out, lengths, mask, wms, n_rec), wms
        if fixed:
            return out, wms
        return ((out, lengths, mask) if self.return_mask else (out, lengths)), wms

    # ------------------------------------------------------------------ collate
    def _collate_tree(self, run: _Run, g: int, payload_bytes: int, copy):
        """A PACK_TREE slot (loader/tree.py) -> the sample structure, leaves on the device."""
        from . import tree

        desc, data = tree.descriptor(run.ring.payload_view(g))
        fdt = self.dtype if self.dtype is not None and self.dtype.is_floating_point else None
        if self.device.type == "cuda":
            block = torch.empty(payload_bytes, dtype=torch.uint8, device=self.device)
            copy(block)
        else:
            block = torch.frombuffer(run.ring.payload_view(g), dtype=torch.uint8, count=payload_bytes).clone()
        return tree.unpack(desc, data, block, fdt)

    def _collate(self, run: _Run, g: int, summ, wms):
        n_rows, _flags, payload_bytes, voff, max_len, total, _w, kind, src_code = summ
        if kind == core().PACK_TREE:
            def copy(block):
                run.engine.copy_raw(g, _stream_ptr(self.device), 0, block.data_ptr(), payload_bytes)
            out = self._collate_tree(run, g, payload_bytes, copy)
            if run.engine is None:
                run.ring.main_release(g)
            if self.return_info:
                return KafkaBatch(out, None, None, wms, sum(w[3] for w in wms))
            return out
        fixed = kind == core().PACK_FIXED
        if src_code >= 0:
            src_dt = CODE_DTYPE[src_code]
            shape = tuple(run.ring.slot_sample(g)[1]) if fixed else None
        else:
            s = self.schema
            src_dt = s.dtype if kind != core().PACK_JSON_F32 else torch.float32
            shape = tuple(s.shape) if fixed else None
        dst_dt = self._out_dtype(src_dt)
        if (dst_dt in FLOAT_DTYPES) != (src_dt in FLOAT_DTYPES) and src_dt in FLOAT_DTYPES:
            raise TypeError(f"cannot collate {src_dt} records to {dst_dt}")
        dev = self.device
        lengths = mask = ext = None
        if fixed:
            x_off, nx = run.ring.slot_extras(g)
            if nx:  # record fields beside the values: [nx, rows] int64 at x_off (read before the slot is released)
                ext = torch.empty((nx, n_rows), dtype=torch.int64, device=dev)
                if run.engine is not None:
                    run.engine.copy_raw(g, _stream_ptr(dev), int(x_off), ext.data_ptr(), nx * n_rows * 8)
                else:
                    ext.copy_(torch.frombuffer(run.ring.payload_view(g), dtype=torch.int64, count=nx * n_rows,
                                               offset=int(x_off)).view(nx, n_rows))
            row = int(max_len) if max_len else 1
            out = torch.empty((n_rows, *shape), dtype=dst_dt, device=dev)
            prm = self._norm_params(row)
            if run.engine is not None:
                shift, scale = (prm[0].data_ptr(), prm[1].data_ptr()) if prm is not None else (0, 0)
                run.engine.collate_fixed(g, _stream_ptr(dev), voff, DTYPE_CODE[src_dt],
                                         out.data_ptr(), DTYPE_CODE[dst_dt], n_rows, row, shift, scale)
            else:
                view = run.ring.payload_view(g)
                src = torch.frombuffer(view, dtype=src_dt, count=n_rows * row, offset=voff).view(n_rows, *shape)
                if prm is None and dst_dt == src_dt:
                    # one memcpy: Tensor.copy_ would split 256 KiB over the intra-op threads, which
                    # contend with the spinning workers for the same cores (~0.3-0.8 ms per batch)
                    ctypes.memmove(out.data_ptr(), src.data_ptr(), out.numel() * out.element_size())
                elif prm is None:
                    out.copy_(src)
                else:
                    out.copy_(((src.reshape(n_rows, row).float() - prm[0]) * prm[1]).to(dst_dt).view(out.shape))
                run.ring.main_release(g)
        else:
            L = self.pad_to if self.pad_to is not None else int(max_len)
            if self.pad_to is None and self.pad_multiple > 1:
                L = (L + self.pad_multiple - 1) // self.pad_multiple * self.pad_multiple
            out = torch.empty((n_rows, L), dtype=dst_dt, device=dev)
            lengths = torch.empty(n_rows, dtype=torch.int64, device=dev)
            mask = torch.empty((n_rows, L), dtype=torch.bool, device=dev) if self.return_mask else None
            if run.engine is not None:
                run.engine.collate_varlen(g, _stream_ptr(dev), voff, DTYPE_CODE[src_dt],
                                          out.data_ptr(), DTYPE_CODE[dst_dt], n_rows, L, float(self.pad_value),
                                          lengths.data_ptr(), mask.data_ptr() if mask is not None else 0)
            else:
                from ..ops.collate import reference_varlen

                view = run.ring.payload_view(g)
                offs = torch.frombuffer(view, dtype=torch.int32, count=n_rows + 1).clone()
                vals = torch.frombuffer(view, dtype=src_dt, count=int(total), offset=voff).clone() if total else \
                    torch.empty(0, dtype=src_dt)
                res = reference_varlen(offs, vals, dst_dt, L, self.pad_value, self.return_mask)
                out.copy_(res[0])
                lengths.copy_(res[1])
                if mask is not None:
                    mask.copy_(res[2])
                run.ring.main_release(g)
        n_rec = sum(w[3] for w in wms)
        if self.return_info:
            return KafkaBatch(out, lengths, mask, wms, n_rec)
        if fixed:
            return out if ext is None else self._with_fields(out, ext)
        return (out, lengths, mask) if self.return_mask else (out, lengths)

    def _with_fields(self, out, ext):
        """(values, fields...) in the order the schema added them (native columns: key first)."""
        order = self.schema.column_order()
        return (out, *(ext[i] for i in order))

    def _norm_params(self, row: int):
        if self.normalize is None:
            return None
        if self._norm is None or self._norm[0].numel() != row:
            self._norm = normalize_params(self.normalize, row, self.device)
        return self._norm

    # ------------------------------------------------------------------ observability
    def ring_occupancy(self) -> dict:
        """Slots of the live iteration's ring by state: ``ready`` (published by a worker, not yet
        taken), ``inflight`` (taken by the main process: staged, collated ahead or still read by
        the GPU), ``filling`` and ``free``; ``prefilled`` = ready + inflight, the batches a timed
        region starting now would not have to wait for."""
        run = self._run
        if run is None or run.closed:
            return {"free": 0, "filling": 0, "ready": 0, "inflight": 0, "prefilled": 0, "n_slots": 0}
        free, filling, ready, inflight = run.ring.slot_states()
        return {"free": free, "filling": filling, "ready": ready, "inflight": inflight,
                "prefilled": ready + inflight, "n_slots": run.ring.n_slots}

    def reset_stats(self) -> None:
        """Zeroes the loader's counters (and the native driver's) -- e.g. after warm-up."""
        self.stats.reset()
        run = self._run
        if run is not None and run.driver is not None and not run.closed:
            run.driver.reset_stats()

    def stats_summary(self) -> dict:
        """Counters so far, including the native driver's (commits, worker fill times, blocking)."""
        run = self._run
        if run is not None and run.driver is not None and not run.closed:
            self._absorb_driver_stats(run.driver)
        return self.stats.summary()

    def close(self) -> None:
        if self._run is not None:
            self._run.close()
            self._run = None
        for br in reversed(getattr(self, "_bridges", [])):  # forwards the last commits, then drops replicas
            br.close()
        self._bridges = []

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
