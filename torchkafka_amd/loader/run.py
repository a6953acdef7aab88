"""One DeviceLoader iteration's resources: the pinned ring, the worker processes (or the packer
thread), the HIP engine and the native step driver.

``_Run`` is built when an iteration starts and closed when it ends: it forks the workers before
HIP is touched in this process, then creates the engine / driver and applies the loader's plan
(mirror, direct, decode-ahead, coalescing, command queue).  The reference has no equivalent: its
DataLoader workers are torch's, each with a kafka-python consumer
(/root/reference/src/kafka_dataset.py:147-171, /root/reference/src/auto_commit.py:20-66).
"""
from __future__ import annotations

import gc
import logging
import multiprocessing as mp
import os
import threading
import time
import uuid
from collections import deque
from typing import TYPE_CHECKING

import torch

from ..ops.native import core, hip
from ..utils import topology
from .worker import worker_main

if TYPE_CHECKING:
    from .device_loader import DeviceLoader

log = logging.getLogger("torchkafka_amd.loader.device_loader")


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
        self.mirror = False  # the HBM mirror is on for this iteration (PathPlan.mirror, RCCL aside)
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
                else:
                    # HIP gives a process GPU_MAX_HW_QUEUES (4) hardware queues and binds streams to
                    # them round-robin: the user's stream, torch's NCCL stream (a DDP job's gradient
                    # all-reduce), the RCCL lockstep's stream and the copy streams each keep one, the
                    # decode streams take what is left (at most 3, at least 1) -- so a collective
                    # waiting for the other ranks never sits in front of a decode kernel those ranks'
                    # progress depends on, nor a decode kernel in front of the gradient all-reduce
                    n = L._decode_streams_fitting(int(self.engine.copy_streams()))
                    if n != int(self.engine.decode_streams()):
                        self.engine.set_decode_streams(n)
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
                # The mirror keeps its two copy streams under the RCCL lockstep too (round 4 gave it
                # one there, to leave the hardware queues to the decode and RCCL streams): one SDMA
                # stream cannot keep ahead of the decode -- fixed-width 25 M rec/s even without the
                # lockstep, against 48-50 M with two; JSON under the lockstep 48.5-51.6 M with two,
                # 32.8 M from the pinned logs (profiles/r05_s35_mirror_rccl).
                # Fixed-width decode splits a segment over workgroups from HBM, which is kept to a mirror
                # whose launches wait for copies in flight: the no-wait policy with split segments failed
                # the device CRC check at four ranks on one GPU (profiles/r06_s21, r06_s23; N = 1 dma
                # block 47.7-48.0 M rec/s waiting against 41.1-45.5 M not).  JSON / var-len decode keep
                # one workgroup per segment and the no-wait policy (round 4: config 4 waits cost it).
                self.mirror = L.plan.mirror
                if self.mirror:
                    fixed = not (L.plan.json_span or L.plan.var_span)
                    self.driver.enable_mirror(int(L.tuning.mirror_chunk_mib) << 20, int(L.tuning.mirror_chunks), 0,
                                              1 if fixed else 0)
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
