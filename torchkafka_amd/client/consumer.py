"""KafkaConsumer over the synthetic broker.

A kafka-python 2.0.2 compatible subset: the constructor, configuration keys
and defaults, iteration semantics (``consumer_timeout_ms``), ``poll``,
``commit`` (sync, requires ``group_id``), ``close(autocommit=...)``,
subscription with consumer-group range assignment and rebalances, manual
``assign``, seeking and offset queries.  The reference builds exactly one of
these per process (kafka_dataset.py:206) and relies on its iteration and
``commit()``; everything the reference touches behaves as in kafka-python.

Additions for the framework (not in kafka-python):
  * ``_fetcher``: the native fetch/decode core used by the loader fast path;
  * ``_idle_hooks``: callbacks run while iteration waits for records, so a
    worker can apply commit requests on idle partitions (fixes reference D8);
  * ``_revoke_hooks``: callbacks run when the group takes this member's partitions away, before
    the user's ``ConsumerRebalanceListener.on_partitions_revoked`` -- the loaders commit what the
    user finished there, so the listener sees those offsets committed;
  * ``assign_shard``: deterministic rank/worker partition sharding (N3);
  * fork detection: using a consumer in a process other than the one that
    created it raises instead of silently sharing state (reference D7).
"""
from __future__ import annotations

import abc
import copy
import itertools
import logging
import os
import time
from collections import deque

from typing import Callable, Iterable

from ..broker.synthetic import open_broker, resolve_url
from ..ops.native import core
from ..parallel.sharding import shard_partitions
from .errors import (
    CommitFailedError, IllegalStateError, KafkaConfigurationError, KafkaError, NoOffsetForPartitionError,
    OffsetOutOfRangeError,
)
from .records import ConsumerRecord, OffsetAndMetadata, OffsetAndTimestamp, TopicPartition

_getpid = os.getpid
log = logging.getLogger(__name__)

# This process's pid, refreshed in every forked child: the per-record fork check in __next__ is an
# int compare instead of a getpid() system call (0.4 us a record at BASELINE config 1's rates).
_PID = [os.getpid()]
os.register_at_fork(after_in_child=lambda: _PID.__setitem__(0, os.getpid()))


class ConsumerRebalanceListener(abc.ABC):
    """kafka-python's rebalance callback interface (``kafka.ConsumerRebalanceListener``), passed to
    :meth:`KafkaConsumer.subscribe`.  Eager semantics, as kafka-python 2.0.2: before every
    (re)join the member gives up its whole assignment -- ``on_partitions_revoked`` with it (an
    empty set before the first join) -- and ``on_partitions_assigned`` receives the complete new
    assignment once the group is stable again.  Both run in the thread that polls the consumer;
    an exception they raise is logged, not propagated (kafka-python's coordinator does the same)."""

    @abc.abstractmethod
    def on_partitions_revoked(self, revoked):
        """``revoked``: set of TopicPartition this member owned until now."""

    @abc.abstractmethod
    def on_partitions_assigned(self, assigned):
        """``assigned``: set of TopicPartition this member owns from now on."""

_GROUP_STABLE = 2


class CommitFuture:
    """Resolved future returned by ``commit_async`` (kafka-python ``Future`` subset)."""

    is_done = True

    def __init__(self):
        self.exception = None
        self.value = None

    def succeeded(self) -> bool:
        return self.exception is None

    def failed(self) -> bool:
        return self.exception is not None

    def add_callback(self, fn, *args, **kwargs) -> "CommitFuture":
        if self.exception is None:
            fn(*args, self.value, **kwargs)
        return self

    def add_errback(self, fn, *args, **kwargs) -> "CommitFuture":
        if self.exception is not None:
            fn(*args, self.exception, **kwargs)
        return self

    def get(self, timeout=None):
        if self.exception is not None:
            raise self.exception
        return self.value


class KafkaConsumer:
    """Consume records from the synthetic broker with kafka-python's API."""

    DEFAULT_CONFIG = {
        "bootstrap_servers": "localhost",
        "client_id": "kafka-python-2.0.2",
        "group_id": None,
        "key_deserializer": None,
        "value_deserializer": None,
        "fetch_max_wait_ms": 500,
        "fetch_min_bytes": 1,
        "fetch_max_bytes": 52428800,
        "max_partition_fetch_bytes": 1 * 1024 * 1024,
        "request_timeout_ms": 305000,
        "retry_backoff_ms": 100,
        "reconnect_backoff_ms": 50,
        "reconnect_backoff_max_ms": 1000,
        "max_in_flight_requests_per_connection": 5,
        "auto_offset_reset": "latest",
        "enable_auto_commit": True,
        "auto_commit_interval_ms": 5000,
        "default_offset_commit_callback": lambda offsets, response: True,
        "check_crcs": True,
        "metadata_max_age_ms": 5 * 60 * 1000,
        "partition_assignment_strategy": None,
        "max_poll_records": 500,
        "max_poll_interval_ms": 300000,
        "session_timeout_ms": 10000,
        "heartbeat_interval_ms": 3000,
        "receive_buffer_bytes": None,
        "send_buffer_bytes": None,
        "socket_options": None,
        "consumer_timeout_ms": float("inf"),
        "security_protocol": "PLAINTEXT",
        "ssl_context": None,
        "ssl_check_hostname": True,
        "ssl_cafile": None,
        "ssl_certfile": None,
        "ssl_keyfile": None,
        "ssl_crlfile": None,
        "ssl_password": None,
        "ssl_ciphers": None,
        "api_version": None,
        "api_version_auto_timeout_ms": 2000,
        "connections_max_idle_ms": 9 * 60 * 1000,
        "metric_reporters": [],
        "metrics_num_samples": 2,
        "metrics_sample_window_ms": 30000,
        "metric_group_prefix": "consumer",
        "selector": None,
        "exclude_internal_topics": True,
        "sasl_mechanism": None,
        "sasl_plain_username": None,
        "sasl_plain_password": None,
        "sasl_kerberos_service_name": "kafka",
        "sasl_kerberos_domain_name": None,
        "sasl_oauth_token_provider": None,
        "legacy_iterator": False,
    }

    def __init__(self, *topics: str, **configs):
        extra = set(configs).difference(self.DEFAULT_CONFIG)
        if extra:
            raise KafkaConfigurationError(f"Unrecognized configs: {extra}")
        self.config = copy.copy(self.DEFAULT_CONFIG)
        self.config.update(configs)
        if self.config["auto_offset_reset"] not in ("earliest", "latest", "none", "smallest", "largest"):
            raise KafkaConfigurationError("auto_offset_reset must be 'earliest', 'latest' or 'none'")
        self._pid = os.getpid()
        self._url = resolve_url(self.config["bootstrap_servers"])
        self._broker = open_broker(self._url)
        self._b = self._broker.native
        self._fetcher = core().Fetcher(self._b, bool(self.config["check_crcs"]))
        self._closed = False
        self._subscription: set[str] = set()
        self._manual = False
        self._assignment: list[int] = []          # global partition indices
        self._paused: set[int] = set()
        self._buffer: deque = deque()
        self._tp_cache: dict[int, TopicPartition] = {}
        self._position: dict[int, int] = {}
        self._idle_hooks: list[Callable[[], None]] = []
        self._revoke_hooks: list[Callable[[], None]] = []
        self._listener: ConsumerRebalanceListener | None = None
        self._revoked = False  # the current assignment was already given up (revoke callbacks ran)
        self._rejoining = False  # rejoined a rebalance round: hand nothing out until it completes
        self._iter_deadline = None
        self._last_auto_commit = time.monotonic()
        # group membership (subscription mode)
        self._g = None if self.config["group_id"] is None else self._b.group_index(self.config["group_id"], True)
        self._member_slot = -1
        self._member_id = 0
        self._generation = 0
        self._group_checked = 0.0
        if topics:
            self.subscribe(topics=topics)

    # ------------------------------------------------------------------ helpers
    def _check_open(self):
        if self._closed:
            raise IllegalStateError("This consumer has already been closed.")
        if os.getpid() != self._pid:
            raise IllegalStateError(
                f"KafkaConsumer created in process {self._pid} is used in process {os.getpid()} "
                "(forked DataLoader worker?). Build the dataset with KafkaDataset.placeholder() and pass "
                "worker_init_fn=KafkaDataset.init_worker(...) so each worker owns its own consumer."
            )

    def _tp(self, pidx: int) -> TopicPartition:
        tp = self._tp_cache.get(pidx)
        if tp is None:
            tp = self._tp_cache[pidx] = self._broker.tp_of(pidx)
        return tp

    def _sync_positions(self) -> None:
        """Consumed (returned-to-user) positions follow kafka-python: they advance as records are
        returned, not as they are fetched.  Partitions without buffered records take the fetch position."""
        buffered = {r[0] for r in self._buffer}
        fetch = self._fetcher.positions()
        self._position = {p: (self._position.get(p, fetch[p]) if p in buffered else fetch[p]) for p in fetch}

    def _pidx(self, tp: TopicPartition) -> int:
        return self._broker.pidx(tp.topic, tp.partition)

    def _reset_position(self, pidx: int) -> int:
        strategy = self.config["auto_offset_reset"]
        if strategy in ("earliest", "smallest"):
            return self._b.log_start_offset(pidx)
        if strategy in ("latest", "largest"):
            return self._b.high_watermark(pidx)
        tp = self._tp(pidx)
        raise NoOffsetForPartitionError(f"NoOffsetForPartitionError: {tp}")

    def _initial_position(self, pidx: int) -> int:
        if self._g is not None:
            off, _ = self._b.committed(self._g, pidx)
            if off >= 0:
                lo, hi = self._b.log_start_offset(pidx), self._b.high_watermark(pidx)
                if lo <= off <= hi:
                    return off
        return self._reset_position(pidx)

    def _call_listener(self, which: str, pidxs) -> None:
        if self._listener is None:
            return
        tps = {self._tp(p) for p in pidxs}
        try:
            getattr(self._listener, which)(tps)
        except Exception:  # noqa: BLE001 - kafka-python logs a failing user listener and carries on
            what = "revocation" if which == "on_partitions_revoked" else "assignment"
            log.exception("User provided listener %s for group %s failed on partition %s", self._listener,
                          self.config["group_id"], what)

    def _revoke(self, owned=None) -> None:
        """This member is about to (re)join: what the user finished is committed (the loaders'
        ``_revoke_hooks``), then the listener is told the whole assignment is gone (eager
        protocol, kafka-python's ``_on_join_prepare``).  Once per rebalance."""
        if self._revoked:
            return
        self._revoked = True
        owned = self._assignment if owned is None else owned
        for hook in list(self._revoke_hooks):
            try:
                hook()
            except Exception:  # noqa: BLE001 - a failed commit is logged, as any other (B14)
                log.exception("commit before partition revocation failed")
        self._call_listener("on_partitions_revoked", owned)

    def _assigned(self, pidxs) -> None:
        self._revoked = False
        self._call_listener("on_partitions_assigned", pidxs)

    def _group_tick(self) -> None:
        """Group maintenance without waiting (a loader's background thread, while the consumer is
        otherwise idle): answers a rebalance round -- commit hooks, revoke callback, rejoin -- and
        takes the new assignment once the group is stable.  kafka-python leaves this to poll();
        a DataLoader worker parked on its index queue would then stall the whole group until the
        rebalance timeout."""
        if self._closed or self._manual or not self._subscription or self._g is None or self._pid != _getpid():
            return
        self._ensure_group(block=False)

    def _set_assignment(self, pidxs: Iterable[int]) -> None:
        pidxs = sorted(set(pidxs))
        old = self._fetcher.positions()
        positions = [old[p] if p in old else self._initial_position(p) for p in pidxs]
        self._fetcher.assign(pidxs, positions)
        for p in pidxs:
            if p in self._paused:
                self._fetcher.pause(p, True)
        # drop buffered records of revoked partitions
        if self._buffer:
            keep = set(pidxs)
            self._buffer = deque(r for r in self._buffer if r[0] in keep)
        self._assignment = pidxs
        self._sync_positions()

    def _ensure_group(self, block: bool = True) -> None:
        """Joins / follows the consumer group (subscription mode).  kafka-python's coordinator poll."""
        if self._manual or not self._subscription:
            return
        if self._g is None:
            # no group: kafka-python-style standalone subscription gets every partition
            if not self._assignment:
                pidxs = []
                for t in sorted(self._subscription):
                    _, n, first = self._broker.topic(t)
                    pidxs += range(first, first + n)
                self._set_assignment(pidxs)
            return
        if self._member_slot < 0:
            self._revoke()  # kafka-python calls it before every join, the first one included
            topics = [self._broker.topic(t)[0] for t in sorted(self._subscription)]
            self._member_slot = self._b.join_group(self._g, topics, int(self.config["session_timeout_ms"]),
                                                   int(self.config["max_poll_interval_ms"]))
            self._member_id = self._b.member_id(self._g, self._member_slot)
        gen, state, active, assignment = self._b.poll_group(self._g, self._member_slot, self._member_id)
        if not active:
            # evicted (max_poll_interval exceeded or broker decided): rejoin
            self._revoke()
            self._member_slot = -1
            self._assignment = []
            self._fetcher.assign([], [])
            self._buffer.clear()
            self._position = {}
            return self._ensure_group()
        if state != _GROUP_STABLE:
            self._revoke()  # a rebalance is under way: give the partitions up (commits first)
            # rejoin: the coordinator reassigns once every member did (or at the rebalance timeout).
            # Nothing more is handed out until then (_rejoining); the fetch positions stay, so a
            # partition the next generation gives back to this member resumes where it was -- it
            # had no other owner in between -- and others start at the group's committed offset.
            self._b.rejoin_group(self._g, self._member_slot, self._member_id)
            self._rejoining = True
            # kafka-python joins the group synchronously (ensure_active_group blocks):
            # wait out the initial rebalance delay instead of returning an empty assignment
            if not block:
                return
            deadline = time.monotonic() + 60.0
            while state != _GROUP_STABLE and time.monotonic() < deadline:
                time.sleep(0.005)
                # idempotent; also answers a round that started while this member waited
                self._b.rejoin_group(self._g, self._member_slot, self._member_id)
                gen, state, active, assignment = self._b.poll_group(self._g, self._member_slot, self._member_id)
                if not active:
                    return self._ensure_group()
            if state != _GROUP_STABLE:
                return
        if gen != self._generation:
            self._revoke()  # the rebalance completed between two polls: revoke before the new assignment
            prev, self._generation = self._generation, gen
            old = set(self._assignment)
            # revoked partitions restart from committed offsets when re-acquired; one this member
            # keeps into the very next generation had no other owner: it resumes where it was
            keep_positions = ({p: pos for p, pos in self._fetcher.positions().items() if p in assignment}
                              if gen == prev + 1 else {})
            pidxs = sorted(assignment)
            positions = [keep_positions[p] if p in keep_positions else self._initial_position(p) for p in pidxs]
            self._fetcher.assign(pidxs, positions)
            if self._buffer:
                keep = set(pidxs)
                self._buffer = deque(r for r in self._buffer if r[0] in keep)
            self._assignment = pidxs
            self._sync_positions()
            if set(pidxs) != old:
                log.debug("group %s generation %d assignment %s", self.config["group_id"], gen,
                          [self._tp(p) for p in pidxs])
            self._rejoining = False
            self._assigned(pidxs)

    def _fetch_into_buffer(self, max_records: int) -> int:
        tps = self._tp_cache
        for p in self._assignment:
            if p not in tps:
                self._tp(p)
        try:
            recs = self._fetcher.poll_consumer_records(max_records, ConsumerRecord, tps)
        except OffsetOutOfRangeError:
            for p in self._assignment:
                lo, hi = self._b.log_start_offset(p), self._b.high_watermark(p)
                pos = self._fetcher.position(p)
                if pos is not None and not lo <= pos <= hi:
                    self._fetcher.seek(p, self._reset_position(p))
                    self._position[p] = self._fetcher.position(p)
            recs = self._fetcher.poll_consumer_records(max_records, ConsumerRecord, tps)
        kd, vd = self.config["key_deserializer"], self.config["value_deserializer"]
        if kd is not None or vd is not None:
            # kafka-python deserializes while parsing fetched records (before iteration)
            recs = [(p, r._replace(key=kd(r.key) if kd is not None and r.key is not None else r.key,
                                   value=vd(r.value) if vd is not None and r.value is not None else r.value))
                    for p, r in recs]
        self._buffer.extend(recs)
        return len(recs)

    def _make_record(self, pidx: int, r: ConsumerRecord) -> ConsumerRecord:
        self._position[pidx] = r.offset + 1
        return r

    def _maybe_auto_commit(self) -> None:
        if self.config["enable_auto_commit"] and self._g is not None:
            now = time.monotonic()
            if (now - self._last_auto_commit) * 1000 >= self.config["auto_commit_interval_ms"]:
                self._last_auto_commit = now
                try:
                    self.commit()
                except CommitFailedError:
                    log.warning("Auto offset commit failed")

    # ------------------------------------------------------------------ subscription API
    def subscribe(self, topics=(), pattern=None, listener=None) -> None:
        self._check_open()
        if self._manual:
            raise IllegalStateError("Subscription to topics, partitions and pattern are mutually exclusive")
        if listener is not None and not isinstance(listener, ConsumerRebalanceListener):
            raise TypeError("listener must be a ConsumerRebalanceListener")
        self._listener = listener
        if pattern is not None:
            import re

            rx = re.compile(pattern)
            topics = [t for t in self._broker.topics() if rx.match(t)]
        if isinstance(topics, str):
            topics = [topics]
        for t in topics:
            self._broker.topic(t)  # raises for unknown topics
        self._subscription = set(topics)
        if self._member_slot >= 0:
            self._b.leave_group(self._g, self._member_slot, self._member_id)
            self._member_slot = -1
        self._assignment = []
        self._fetcher.assign([], [])

    def subscription(self):
        return set(self._subscription) if self._subscription else None

    def unsubscribe(self) -> None:
        self._check_open()
        if self._member_slot >= 0:
            self._b.leave_group(self._g, self._member_slot, self._member_id)
            self._member_slot = -1
        self._subscription = set()
        self._manual = False
        self._assignment = []
        self._fetcher.assign([], [])
        self._buffer.clear()

    def assign(self, partitions) -> None:
        self._check_open()
        if self._subscription:
            raise IllegalStateError("Subscription to topics, partitions and pattern are mutually exclusive")
        self._manual = True
        self._set_assignment(self._pidx(tp) for tp in partitions)

    def assign_shard(self, topics, rank: int, world_size: int, worker_id: int = 0, num_workers: int = 1) -> list:
        """Static (rank, worker) sharding of every partition of ``topics``.

        Partition p goes to rank ``p % world_size`` and, inside it, to worker
        ``(p // world_size) % num_workers``.  Replaces any subscription.
        """
        if isinstance(topics, str):
            topics = [topics]
        if self._subscription:
            self.unsubscribe()
        tps = []
        for t in topics:
            n = self._broker.topic(t)[1]
            tps += [TopicPartition(t, p) for p in shard_partitions(n, rank, world_size, worker_id, num_workers)]
        self._manual = True
        self._set_assignment(self._pidx(tp) for tp in tps)
        return tps

    def assignment(self) -> set:
        self._ensure_group()
        return {self._tp(p) for p in self._assignment}

    # ------------------------------------------------------------------ positions
    def position(self, partition: TopicPartition) -> int:
        self._check_open()
        self._ensure_group()
        p = self._pidx(partition)
        if p not in self._assignment:
            raise IllegalStateError(f"Partition {partition} is not assigned")
        return self._position.get(p, self._fetcher.position(p))

    def seek(self, partition: TopicPartition, offset: int) -> None:
        self._check_open()
        if offset < 0:
            raise ValueError("offset must be >= 0")
        p = self._pidx(partition)
        self._fetcher.seek(p, int(offset))
        self._buffer = deque(r for r in self._buffer if r[0] != p)
        self._position[p] = int(offset)

    def seek_to_beginning(self, *partitions) -> None:
        for tp in partitions or self.assignment():
            self.seek(tp, self._b.log_start_offset(self._pidx(tp)))

    def seek_to_end(self, *partitions) -> None:
        for tp in partitions or self.assignment():
            self.seek(tp, self._b.high_watermark(self._pidx(tp)))

    def committed(self, partition: TopicPartition, metadata: bool = False):
        if self._g is None:
            raise AssertionError("Requires group_id")
        off, meta = self._b.committed(self._g, self._pidx(partition))
        if off < 0:
            return None
        return OffsetAndMetadata(off, meta) if metadata else off

    def beginning_offsets(self, partitions) -> dict:
        return {tp: self._b.log_start_offset(self._pidx(tp)) for tp in partitions}

    def end_offsets(self, partitions) -> dict:
        return {tp: self._b.high_watermark(self._pidx(tp)) for tp in partitions}

    def offsets_for_times(self, timestamps: dict) -> dict:
        """``{tp: ts_ms}`` -> ``{tp: OffsetAndTimestamp | None}``: earliest offset whose timestamp is >= ts."""
        out = {}
        for tp, ts in timestamps.items():
            if int(ts) < 0:
                raise ValueError(f"The target time for partition {tp} is {ts}. It should be non-negative.")
            off, rts = self._b.offset_for_time(self._pidx(tp), int(ts))
            out[tp] = OffsetAndTimestamp(off, rts) if off >= 0 else None
        return out

    def highwater(self, partition: TopicPartition) -> int:
        return self._b.high_watermark(self._pidx(partition))

    def partitions_for_topic(self, topic: str):
        return self._broker.partitions_for(topic) if self._broker.has_topic(topic) else None

    def topics(self) -> set:
        return set(self._broker.topics())

    def pause(self, *partitions) -> None:
        for tp in partitions:
            p = self._pidx(tp)
            self._paused.add(p)
            if p in self._assignment:
                self._fetcher.pause(p, True)

    def resume(self, *partitions) -> None:
        for tp in partitions:
            p = self._pidx(tp)
            self._paused.discard(p)
            if p in self._assignment:
                self._fetcher.pause(p, False)

    def paused(self) -> set:
        return {self._tp(p) for p in self._paused}

    # ------------------------------------------------------------------ fetching
    def poll(self, timeout_ms: int = 0, max_records: int | None = None, update_offsets: bool = True) -> dict:
        """Returns ``{TopicPartition: [ConsumerRecord]}``; waits up to ``timeout_ms`` for data.

        ``update_offsets=False`` peeks: the records stay buffered and positions do not move, so the next
        ``poll``/``next`` returns them again (kafka-python's semantics).
        """
        self._check_open()
        max_records = max_records or self.config["max_poll_records"]
        deadline = time.monotonic() + timeout_ms / 1000.0
        backoff = 0.0002
        while True:
            self._ensure_group()
            self._maybe_auto_commit()
            if not self._buffer:
                self._fetch_into_buffer(max_records)
            if self._buffer:
                out: dict = {}
                if not update_offsets:
                    for _, r in itertools.islice(self._buffer, max_records):
                        out.setdefault(TopicPartition(r.topic, r.partition), []).append(r)
                    return out
                for _ in range(min(max_records, len(self._buffer))):
                    pidx, r = self._buffer.popleft()
                    rec = self._make_record(pidx, r)
                    out.setdefault(TopicPartition(rec.topic, rec.partition), []).append(rec)
                return out
            now = time.monotonic()
            if now >= deadline:
                return {}
            for hook in self._idle_hooks:
                hook()
            time.sleep(min(backoff, max(0.0, deadline - now)))
            backoff = min(backoff * 2, 0.01)

    def __iter__(self):
        return self

    def __next__(self) -> ConsumerRecord:
        """Blocks for the next record; StopIteration after ``consumer_timeout_ms`` without one."""
        buf = self._buffer
        if buf and not self._rejoining and not self._closed and self._pid == _PID[0]:
            pidx, r = buf.popleft()  # hot path: one record from the fetched buffer
            self._position[pidx] = r[2] + 1
            return r
        self._check_open()
        timeout = self.config["consumer_timeout_ms"]
        deadline = None if timeout == float("inf") else time.monotonic() + timeout / 1000.0
        backoff = 0.0002
        while True:
            if self._rejoining:
                self._ensure_group()  # a rebalance round this member rejoined from a background tick
            if self._buffer and not self._rejoining:
                pidx, r = self._buffer.popleft()
                return self._make_record(pidx, r)
            self._ensure_group()
            self._maybe_auto_commit()
            if self._fetch_into_buffer(self.config["max_poll_records"]):
                continue
            now = time.monotonic()
            if deadline is not None and now >= deadline:
                raise StopIteration
            for hook in self._idle_hooks:
                hook()
            sleep = backoff if deadline is None else min(backoff, max(0.0, deadline - now))
            time.sleep(sleep)
            backoff = min(backoff * 2, 0.01)

    # ------------------------------------------------------------------ commits
    def _consumed_offsets(self) -> dict[int, int]:
        """Positions of assigned partitions, excluding records still in the iteration buffer."""
        return {p: self._position.get(p, 0) for p in self._assignment}

    def commit(self, offsets: dict | None = None) -> None:
        """Synchronously commits ``offsets`` (default: every consumed position).  Requires group_id."""
        self._check_open()
        assert self.config["group_id"] is not None, "Requires group_id"
        if offsets is None and isinstance(self._assignment, list):
            if self._manual or not self._subscription:
                self._b.commit_positions(self._g, -1, 0, 0, self._assignment, self._position)
            else:
                if self._member_slot < 0:
                    raise CommitFailedError("CommitFailedError: consumer is not part of an active group")
                self._b.commit_positions(self._g, self._member_slot, self._member_id, self._generation,
                                         self._assignment, self._position)
            return
        if offsets is None:
            entries = [(p, int(o), "") for p, o in self._consumed_offsets().items()]
        else:
            entries = []
            for tp, om in offsets.items():
                off, meta = (om.offset, om.metadata or "") if isinstance(om, OffsetAndMetadata) else (int(om), "")
                entries.append((self._pidx(tp), int(off), meta))
        if not entries:
            return
        if self._manual or not self._subscription:
            self._b.commit(self._g, -1, 0, 0, entries)
        else:
            if self._member_slot < 0:
                raise CommitFailedError("CommitFailedError: consumer is not part of an active group")
            self._b.commit(self._g, self._member_slot, self._member_id, self._generation, entries)

    def commit_async(self, offsets=None, callback=None) -> "CommitFuture":
        """kafka-python's async commit.  The shared-memory commit takes well under a microsecond, so it runs
        inline; ``callback(offsets, exc_or_none)`` follows and the returned future is already resolved.

        As in kafka-python, the callback receives the ``{TopicPartition: OffsetAndMetadata}`` that was
        committed (the consumed positions when ``offsets`` is None), ``default_offset_commit_callback``
        stands in when no callback is given, and a KafkaError lands in the future instead of raising."""
        fut = CommitFuture()
        if offsets is None:
            self._check_open()
            committed = {self._tp(p): OffsetAndMetadata(o, "") for p, o in self._consumed_offsets().items()}
        else:
            committed = {tp: om if isinstance(om, OffsetAndMetadata) else OffsetAndMetadata(int(om), "")
                         for tp, om in offsets.items()}
        try:
            self.commit(offsets)
        except KafkaError as e:
            fut.exception = e
        else:
            fut.value = committed
        cb = callback if callback is not None else self.config["default_offset_commit_callback"]
        cb(committed, fut.exception)
        return fut

    # ------------------------------------------------------------------ lifecycle
    def close(self, autocommit: bool = True) -> None:
        if self._closed:
            return
        if os.getpid() != self._pid:
            self._closed = True  # inherited by fork: nothing of ours to release here
            return
        try:
            if autocommit and self.config["enable_auto_commit"] and self._g is not None:
                try:
                    self.commit()
                except Exception:  # noqa: BLE001 - kafka-python logs and continues on close
                    log.exception("Auto offset commit failed on close")
            if self._member_slot >= 0:
                self._b.leave_group(self._g, self._member_slot, self._member_id)
                self._member_slot = -1
        finally:
            self._closed = True

    def metrics(self, raw: bool = False) -> dict:
        out = {}
        for p in self._assignment:
            tp = self._tp(p)
            out[f"{tp.topic}-{tp.partition}"] = self._b.partition_stats(p)
        return out

    def bootstrap_connected(self) -> bool:
        return not self._closed

    def __del__(self):
        try:
            if not self._closed and os.getpid() == self._pid and self._member_slot >= 0:
                self._b.leave_group(self._g, self._member_slot, self._member_id)
        except Exception:  # noqa: BLE001
            pass
