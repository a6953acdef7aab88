"""DeviceLoader worker process: consume records and pack batches into pinned ring slots.

One process per worker (forked before the parent touches HIP, or spawned);
it never initialises the GPU.  Two paths:

* **native** (dataset declares a ``schema`` and the consumer is the synthetic
  broker's): one ``Fetcher.fill_slot`` call per batch decodes RecordBatches
  straight out of the broker log, applies the schema's None-skip filter and
  packs values into the slot; no Python per record.
* **generic** (any ``_process``): the reference's per-record loop
  (kafka_dataset.py:156-162) runs unchanged, and the samples are stacked
  directly into the slot's pinned memory (dense) or written as CSR
  (variable-length 1-D samples), with per-partition offset watermarks.

Errors are shipped to the main process in a slot marked SLOT_ERROR.
"""
from __future__ import annotations

import os
import random
import traceback

import numpy as np
import torch

from ..ops.native import core

_DT_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float8_e4m3fn: 3, torch.uint8: 4,
            torch.int8: 5, torch.int32: 6, torch.int64: 7}


class _StopWorker(Exception):
    pass


def _set_worker_info(worker_id: int, num_workers: int, seed: int, dataset) -> None:
    from torch.utils.data._utils import worker as _w

    _w._worker_info = _w.WorkerInfo(id=worker_id, num_workers=num_workers, seed=seed, dataset=dataset)


def _die_with_parent() -> None:
    """A worker never outlives the process that forked it (PR_SET_PDEATHSIG): a main process that
    dies or is killed without closing its loader leaves no worker holding the ring or the broker."""
    try:
        import ctypes
        import signal

        ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGKILL), 0, 0, 0)  # PR_SET_PDEATHSIG
    except (OSError, AttributeError):
        return
    if os.getppid() == 1:  # the parent died before the call
        os._exit(1)


def worker_main(ring, ring_name: str, worker_id: int, num_workers: int, dataset, worker_init_fn, cfg: dict) -> None:
    """Entry point of a DeviceLoader worker process."""
    if ring is None:
        ring = core().Ring.open(ring_name)
    in_process = bool(cfg.get("in_process", False))  # num_workers=0: a thread of the main process
    ring.set_worker_pid(worker_id, os.getpid())
    # spin (µs) on a full sub-ring before sleeping: keeps futex wakes off the main thread's path
    ring.set_worker_spin_ns(int(cfg.get("worker_spin_us", 200)) * 1000)
    spw = ring.slots_per_worker
    state = {"i": 0, "g": None}
    try:
        if not in_process:  # process-wide state belongs to the user in single-process mode
            _die_with_parent()
            torch.set_num_threads(1)
            seed = int(cfg.get("base_seed", 0)) + worker_id
            random.seed(seed)
            torch.manual_seed(seed)
            np.random.seed(seed % (2**32))
            _set_worker_info(worker_id, num_workers, seed, dataset)
            if worker_init_fn is not None:
                worker_init_fn(worker_id)
        consumer = getattr(dataset, "_consumer", None)
        state["consumer"] = consumer
        if consumer is None:
            raise RuntimeError(
                "DeviceLoader worker has no consumer: build the dataset with placeholder() and pass "
                "worker_init_fn=YourDataset.init_worker(topic, ...)")
        if not in_process:
            dataset._worker_id = worker_id
        if cfg["sharding"] == "static" and getattr(consumer, "_bridged_shard", False):
            pass  # a native wire-route consumer: its bridge already mirrors exactly this worker's shard
        elif cfg["sharding"] == "static":
            topics = sorted(consumer.subscription() or [])
            if not topics:
                raise RuntimeError("static sharding needs the consumer to be created with its topics")
            if not hasattr(consumer, "assign_shard"):
                raise RuntimeError("static sharding needs the synthetic-broker consumer; use sharding='group' "
                                   "with a kafka-python consumer (Kafka's group assignment shards partitions)")
            consumer.assign_shard(topics, cfg["rank"], cfg["world_size"], worker_id, num_workers)
        sink = _WorkerSink(cfg.get("commit_table"), worker_id, dataset, consumer, cfg.get("commit_mode") == "sync")
        state["sink"] = sink
        hooks = getattr(consumer, "_revoke_hooks", None)
        if hooks is not None and sink.table is not None:
            # a rebalance takes partitions away: what the user finished is committed first, then the
            # user's ConsumerRebalanceListener hears of the revocation
            hooks.append(sink.serve_once)
        if (cfg["native"] and getattr(consumer, "_fetcher", None) is not None and dataset.schema is not None
                and not cfg.get("process_overridden", False)):
            sink.start_thread()
            _native_loop(ring, worker_id, spw, consumer, dataset.schema, cfg, state)
        else:
            # a `_process` of its own (or a consumer without the native fetcher): the reference's
            # per-record loop, kafka_dataset.py:156-162
            _generic_loop(ring, worker_id, spw, consumer, dataset, cfg, state)
        sink.serve_until_shutdown(ring)
    except _StopWorker:
        sink = state.get("sink")
        if sink is not None:
            sink.serve_once()  # the final commit request may have come with the shutdown
        return
    except BaseException:  # noqa: BLE001 - everything goes to the main process
        msg = f"Caught exception in DeviceLoader worker {worker_id} (pid {os.getpid()}):\n{traceback.format_exc()}"
        try:
            g = state["g"]
            if g is None:
                if not ring.worker_acquire(worker_id, state["i"], 10000):
                    return
                g = ring.gslot(worker_id, state["i"])
            ring.set_slot(g, 0, 0, 0, 0, 0, 0, 0, 0, [])
            ring.set_error(g, msg)
            ring.worker_publish(g)
        except Exception:  # noqa: BLE001
            pass
    finally:
        # a native wire-route consumer: forward what it committed before this process ends (its
        # bridge's committer thread runs every few ms; the last commit must not be lost).  In
        # single-process mode the consumer is the dataset's: it lives on with the dataset.
        for br in [] if in_process else reversed(getattr(state.get("consumer"), "_bridges", None) or []):
            try:
                br.close()
            except Exception:  # noqa: BLE001 - logged by the bridge
                pass


class _WorkerSink:
    """commit_sink='worker': this worker's consumer commits the offsets the main process
    published for its partitions (loader/commit_channel.py WatermarkTable) -- as a group member
    when the consumer joined a group, through kafka-python when that is the consumer -- with the
    reference's worker log messages and CommitFailedError handling (kafka_dataset.py:124-143)."""

    def __init__(self, table, worker_id, dataset, consumer, sync: bool = False):
        import threading

        self.table, self.w, self.ds, self.consumer = table, worker_id, dataset, consumer
        self.sync = sync
        self.seen = 0
        self.committed: dict = {}
        self.lock = threading.Lock()   # the consumer is used by one thread at a time
        self.local_tps: list = []      # generic loop without a broker: local id -> TopicPartition
        self._thread = None

    def tp_of(self, pidx: int):
        broker = getattr(self.consumer, "_broker", None)
        if broker is not None:
            return broker.tp_of(pidx)
        return self.local_tps[pidx & 0xFFFF]

    def serve_once(self) -> None:
        t = self.table
        if t is None:
            return
        seq = t.requested(self.w)
        if seq <= self.seen:
            return
        from ..client.records import OffsetAndMetadata

        offsets = {}
        for pidx, off in t.entries(self.w):
            if off > self.committed.get(pidx, -1):
                offsets[pidx] = off
        if offsets:
            with self.lock:
                self.ds._do_commit({self.tp_of(p): OffsetAndMetadata(o, "") for p, o in offsets.items()})
                if self.sync:  # commit='sync': the coordinator answered before the request is acked
                    for br in getattr(self.consumer, "_bridges", None) or []:
                        br.commit_sync()
            # a failed commit (rebalance) is logged and not retried, as in the reference (B14)
            self.committed.update(offsets)
        self.seen = seq
        t.ack(self.w, seq)

    def start_thread(self) -> None:
        """Native loop: the fill runs in C++ without the GIL; commits are served beside it."""
        if self.table is None or self._thread is not None:
            return
        import threading
        import time

        def run():
            while True:
                time.sleep(0.001)
                try:
                    self.serve_once()
                except Exception:  # noqa: BLE001 - logged; the next request retries
                    import logging

                    logging.getLogger(__name__).exception("commit on worker %d failed", self.w)

        self._thread = threading.Thread(target=run, name="torchkafka-worker-commit", daemon=True)
        self._thread.start()

    def serve_until_shutdown(self, ring) -> None:
        """After end of stream: keep committing what the user finishes until the loader closes."""
        if self.table is None:
            return
        import time

        while not ring.is_shutdown():
            self.serve_once()
            time.sleep(0.001)
        self.serve_once()


def _acquire(ring, worker_id: int, state: dict) -> int:
    if not ring.worker_acquire(worker_id, state["i"], -1):
        raise _StopWorker
    g = ring.gslot(worker_id, state["i"])
    state["g"] = g
    return g


def _publish(ring, worker_id: int, spw: int, state: dict) -> None:
    ring.worker_publish(state["g"])
    state["g"] = None
    state["i"] = (state["i"] + 1) % spw


def _consumer_timeout_ms(consumer) -> int:
    t = getattr(consumer, "config", {}).get("consumer_timeout_ms", float("inf"))
    return -1 if t == float("inf") else int(t)


def _native_loop(ring, worker_id, spw, consumer, schema, cfg, state) -> None:
    from ..client.errors import OffsetOutOfRangeError

    kind, elem, row_elems, min_len, max_len, trunc, skip_bad = schema.native_spec()
    extras, key_enc, key_default = schema.extras_spec() if hasattr(schema, "extras_spec") else (0, 0, -1)
    if kind == core().PACK_JSON_F32 and cfg.get("json_device"):
        kind = core().PACK_JSON_TEXT  # frame + copy the text; the gfx950 kernel parses it
    bs = int(cfg["batch_size"])
    timeout = _consumer_timeout_ms(consumer)
    fetcher = consumer._fetcher
    gather = bool(cfg.get("gather")) and kind == core().PACK_FIXED
    span = int(bool(cfg.get("span")) and kind in (core().PACK_FIXED, core().PACK_JSON_TEXT, core().PACK_VARLEN)
               and not gather)
    if span and kind == core().PACK_JSON_TEXT and cfg.get("json_count"):
        span = core().SPAN_JSON_DEV_COUNT  # headers only: the device counts the elements
    # a member of a Kafka group over KafkaBridge replicas: the partitions move with rebalances, and
    # a fill waiting for data returns early when they do
    group_managed = bool(getattr(consumer, "_group_managed", False))
    if group_managed:
        fetcher.watch([br._r for br in consumer._bridges])
    if not fetcher.assigned() and cfg["sharding"] == "static" and not group_managed:
        g = _acquire(ring, worker_id, state)  # nothing to read, ever: end of stream right away
        ring.set_slot(g, 0, core().SLOT_EOS, kind, 0, 0, 0, 0, 0, [])
        _publish(ring, worker_id, spw, state)
        return
    while True:
        g = _acquire(ring, worker_id, state)
        consumer._ensure_group()
        while True:
            if group_managed:
                fetcher.set_watch_base(consumer._seen_epoch)
            try:
                rows, _scanned, timed_out, shut = fetcher.fill_slot(ring, g, kind, elem, row_elems, min_len,
                                                                    max_len, trunc, skip_bad, bs, timeout,
                                                                    gather, span, extras, key_enc, key_default)
                if group_managed and fetcher.last_reassigned:
                    consumer._ensure_group()  # the next fill reads the new assignment
                    if rows == 0:
                        continue  # nothing packed yet: fill this slot from the new partitions
                break
            except OffsetOutOfRangeError:
                # retention moved past a position: reset it like the consumer would and refill this slot
                b = consumer._b
                for p in fetcher.assigned():
                    pos = fetcher.position(p)
                    if not b.log_start_offset(p) <= pos <= b.high_watermark(p):
                        fetcher.seek(p, consumer._reset_position(p))
        if shut:
            raise _StopWorker
        if timed_out:
            ring.set_flags(g, core().SLOT_EOS)
        _publish(ring, worker_id, spw, state)
        if timed_out:
            return


def _generic_loop(ring, worker_id, spw, consumer, dataset, cfg, state) -> None:
    """The reference's per-record loop (kafka_dataset.py:156-162) around ``dataset._process``,
    over ``consumer.poll`` so commit requests are served between polls (kafka-python consumers
    are not thread-safe) and an idle partition never blocks them (D8).  Watermarks carry the
    synthetic broker's partition index, or -- for any other consumer (kafka-python) -- a
    worker-local id of the (topic, partition) that only this worker's commit sink resolves."""
    import time

    bs = int(cfg["batch_size"])
    broker = getattr(consumer, "_broker", None)
    sink = state.get("sink")
    cap = ring.payload_capacity
    samples: list = []
    wm: dict = {}  # pidx -> [first, next, count]
    first_pos: dict = {}
    local: dict = {}
    timeout_ms = _consumer_timeout_ms(consumer)

    def pidx_of(rec):
        if broker is not None:
            return broker.pidx(rec.topic, rec.partition)
        if sink is None or sink.table is None:
            raise RuntimeError("DeviceLoader needs commit_sink='worker' for a consumer other than the synthetic "
                               "broker's")
        key = (rec.topic, rec.partition)
        k = local.get(key)
        if k is None:
            from ..client.records import TopicPartition

            k = local[key] = (worker_id << 16) | len(sink.local_tps)
            sink.local_tps.append(TopicPartition(rec.topic, rec.partition))
        return k

    def flush(eos: bool) -> None:
        g = _acquire(ring, worker_id, state)
        view = ring.payload_view(g)
        wms = [(p, v[0], v[1], v[2]) for p, v in wm.items()]
        if samples and not isinstance(samples[0], torch.Tensor):
            # (features, label), {"x": ..., "y": ...}: one stacked region per leaf (loader/tree.py)
            from . import tree

            nbytes = tree.pack(samples, view, cap)
            ring.set_slot(g, len(samples), core().SLOT_EOS if eos else 0, core().PACK_TREE, nbytes, 0, 0, 0,
                          len(samples), wms)
            ring.set_slot_sample(g, -1, [])
        elif samples:
            s0 = samples[0]
            dt = s0.dtype
            code = _DT_CODE.get(dt)
            if code is None:
                raise TypeError(f"unsupported sample dtype {dt}")
            same = all(s.shape == s0.shape and s.dtype == dt for s in samples)
            esize = s0.element_size()
            if same:
                nbytes = len(samples) * s0.numel() * esize
                if nbytes > cap:
                    raise RuntimeError(f"batch of {nbytes} bytes exceeds the ring slot ({cap}); raise slot_bytes")
                dst = torch.frombuffer(view, dtype=dt, count=len(samples) * s0.numel()).view(len(samples), *s0.shape)
                torch.stack(samples, out=dst)
                ring.set_slot(g, len(samples), core().SLOT_EOS if eos else 0, core().PACK_FIXED, nbytes, 0,
                              s0.numel(), len(samples) * s0.numel(), len(samples), wms)
                ring.set_slot_sample(g, code, list(s0.shape))
            else:
                if any(s.dim() != 1 or s.dtype != dt for s in samples):
                    raise TypeError("DeviceLoader needs equal-shape samples or 1-D variable-length samples")
                n = len(samples)
                voff = (4 * (n + 1) + 255) // 256 * 256
                lens = [s.numel() for s in samples]
                total = sum(lens)
                nbytes = voff + total * esize
                if nbytes > cap:
                    raise RuntimeError(f"batch of {nbytes} bytes exceeds the ring slot ({cap}); raise slot_bytes")
                offs = torch.frombuffer(view, dtype=torch.int32, count=n + 1)
                offs[0] = 0
                offs[1:] = torch.tensor(lens, dtype=torch.int64).cumsum(0).to(torch.int32)
                vals = torch.frombuffer(view, dtype=dt, count=total, offset=voff)
                torch.cat(samples, out=vals)
                ring.set_slot(g, n, core().SLOT_EOS if eos else 0, core().PACK_VARLEN, nbytes, voff, max(lens),
                              total, n, wms)
                ring.set_slot_sample(g, code, [])
        else:
            ring.set_slot(g, 0, core().SLOT_EOS if eos else 0, 0, 0, 0, 0, 0, 0, wms)
        _publish(ring, worker_id, spw, state)
        samples.clear()
        wm.clear()

    last_data = time.monotonic()
    while True:
        if sink is not None:
            sink.serve_once()
        if ring.is_shutdown():
            raise _StopWorker
        with (sink.lock if sink is not None else _nolock):
            polled = consumer.poll(timeout_ms=20, max_records=max(1, bs - len(samples)))
        if not polled:
            if timeout_ms >= 0 and (time.monotonic() - last_data) * 1000.0 >= timeout_ms:
                break  # consumer_timeout_ms without records: end of stream, as the consumer iterator does
            continue
        last_data = time.monotonic()
        for _tp, records in polled.items():
            for record in records:
                p = pidx_of(record)
                ent = wm.get(p)
                if ent is None:
                    ent = wm[p] = [first_pos.get(p, record.offset), record.offset + 1, 0]
                ent[1] = record.offset + 1
                ent[2] += 1
                first_pos[p] = record.offset + 1
                data = dataset._process(record)
                if data is None:
                    continue
                samples.append(data)
                if len(samples) == bs:
                    flush(False)
    flush(True)


class _NoLock:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_nolock = _NoLock()
