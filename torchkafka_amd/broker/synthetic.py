"""Synthetic Kafka broker: Python façade over ``_tkcore.Broker``.

kafka-python and a Kafka cluster are unavailable here, so the framework ships
its own broker.  It is a real log store -- partitioned append-only logs of
Kafka RecordBatch v2 bytes, committed offsets per (group, partition), consumer
groups with range assignment and generations -- living in shared memory
(``shm://name``) or in a directory (``file:///path``) so committed offsets
survive restarts.  Several processes (loader workers, DDP ranks) open the
same broker by URL.

Fault injection hooks (commit failures, slow/failing partitions, retention)
exist so the reference's failure behaviour can
be tested deterministically.
"""
from __future__ import annotations

import os
import shutil
import threading
import time
from typing import Iterable, Sequence

from ..client.errors import KafkaError, NoBrokersAvailable
from ..client.records import TopicPartition
from ..ops.native import core

SYNTHETIC_SCHEMES = ("shm://", "file://")

# synthetic record kinds understood by the native generator
KIND_FIXED_F32 = 0
KIND_JSON_F32 = 1
KIND_BYTES = 2
KIND_TOKENS_I32 = 3
KIND_VARLEN_F32 = 4
_KINDS = {"fixed_f32": KIND_FIXED_F32, "json_f32": KIND_JSON_F32, "bytes": KIND_BYTES,
          "tokens_i32": KIND_TOKENS_I32, "varlen_f32": KIND_VARLEN_F32}

_cache: dict[tuple[int, str], "SyntheticBroker"] = {}
_cache_lock = threading.Lock()


def is_synthetic_url(servers) -> bool:
    url = _first_server(servers)
    return url is not None and (url.startswith(SYNTHETIC_SCHEMES) or url.startswith("/"))


def _first_server(servers):
    if servers is None:
        return None
    if isinstance(servers, (list, tuple)):
        return servers[0] if servers else None
    return str(servers).split(",")[0].strip()


def resolve_url(servers) -> str:
    """Maps ``bootstrap_servers`` to a synthetic broker URL.

    Synthetic URLs pass through.  Anything else (``localhost:9092``) resolves
    to ``$TORCHKAFKA_BROKER`` when set, so code written for a real cluster can
    run unchanged against the synthetic broker; otherwise NoBrokersAvailable.
    """
    url = _first_server(servers)
    if url is not None and (url.startswith(SYNTHETIC_SCHEMES) or url.startswith("/")):
        return url
    env = os.environ.get("TORCHKAFKA_BROKER")
    if env:
        return env
    raise NoBrokersAvailable(
        f"NoBrokersAvailable: cannot reach {servers!r}: kafka-python is not installed and "
        "no synthetic broker is configured (use bootstrap_servers='shm://<name>', set TORCHKAFKA_BROKER, or "
        "mirror the cluster with torchkafka.KafkaBridge(servers, topic, group_id=...) and pass bridge.url)"
    )


class SyntheticBroker:
    """Handle on a synthetic broker.  Cheap to share; one per (process, URL) via :func:`open_broker`."""

    def __init__(self, url: str, create: bool = False, *, max_partitions: int = 4096, max_topics: int = 256,
                 max_groups: int = 64, log_capacity: int = 256 << 20, index_capacity: int = 1 << 20,
                 group_initial_rebalance_delay_ms: int = 100):
        self.url = url
        try:
            self._b = core().Broker(url, create, max_topics=max_topics, max_partitions=max_partitions,
                                    max_groups=max_groups, log_capacity=log_capacity,
                                    index_capacity=index_capacity,
                                    group_initial_rebalance_delay_ms=group_initial_rebalance_delay_ms)
        except KafkaError as e:
            if "NoBrokersAvailable" in str(e):
                raise NoBrokersAvailable(str(e)) from None
            raise
        self._topic_cache: dict[str, tuple[int, int, int]] = {}

    # ------------------------------------------------------------ lifecycle
    @classmethod
    def create(cls, url: str, **kw) -> "SyntheticBroker":
        b = cls(url, create=True, **kw)
        with _cache_lock:
            _cache[(os.getpid(), url)] = b
        return b

    @property
    def native(self):
        return self._b

    @property
    def dir(self) -> str:
        return self._b.dir

    def destroy(self) -> None:
        """Removes the broker's files (all topics, offsets).  Other handles become invalid."""
        with _cache_lock:
            for k in [k for k in _cache if k[1] == self.url]:
                del _cache[k]
        shutil.rmtree(self._b.dir, ignore_errors=True)

    # ------------------------------------------------------------ topics
    def create_topic(self, topic: str, num_partitions: int = 1, *, log_capacity: int = 0,
                     index_capacity: int = 0) -> None:
        self._b.create_topic(topic, int(num_partitions), int(log_capacity), int(index_capacity))
        self._topic_cache.pop(topic, None)

    def topic(self, topic: str) -> tuple[int, int, int]:
        """(topic index, n_partitions, first global partition index)."""
        t = self._topic_cache.get(topic)
        if t is None:
            t = self._b.find_topic(topic)
            if t is None:
                raise KafkaError(f"UnknownTopicOrPartitionError: topic {topic!r} does not exist")
            self._topic_cache[topic] = t
        return t

    def has_topic(self, topic: str) -> bool:
        return self._b.find_topic(topic) is not None

    def topics(self) -> list[str]:
        return [t[0] for t in self._b.topics()]

    def partitions_for(self, topic: str) -> set[int]:
        return set(range(self.topic(topic)[1]))

    def pidx(self, topic: str, partition: int) -> int:
        _, n, first = self.topic(topic)
        if not 0 <= partition < n:
            raise KafkaError(f"UnknownTopicOrPartitionError: {topic}-{partition}")
        return first + partition

    def tp_of(self, pidx: int) -> TopicPartition:
        ti, p = self._b.partition_of(pidx)
        return TopicPartition(self._b.topics()[ti][0], p)

    # ------------------------------------------------------------ offsets
    def end_offset(self, topic: str, partition: int) -> int:
        return self._b.high_watermark(self.pidx(topic, partition))

    def beginning_offset(self, topic: str, partition: int) -> int:
        return self._b.log_start_offset(self.pidx(topic, partition))

    def end_offsets(self, topic: str) -> dict[int, int]:
        return {p: self.end_offset(topic, p) for p in range(self.topic(topic)[1])}

    def committed(self, group: str, topic: str, partition: int) -> int | None:
        g = self._b.group_index(group, True)
        off, _ = self._b.committed(g, self.pidx(topic, partition))
        return None if off < 0 else off

    def committed_offsets(self, group: str, topic: str) -> dict[int, int | None]:
        return {p: self.committed(group, topic, p) for p in range(self.topic(topic)[1])}

    def commit_count(self, group: str) -> int:
        return self._b.commit_count(self._b.group_index(group, True))

    def commit(self, group: str, offsets: dict[TopicPartition, int]) -> None:
        """Administrative commit (non-member); fails if the group has active members."""
        g = self._b.group_index(group, True)
        self._b.commit(g, -1, 0, 0, [(self.pidx(tp.topic, tp.partition), int(o), "") for tp, o in offsets.items()])

    def reset_group(self, group: str) -> None:
        self._b.reset_group_offsets(self._b.group_index(group, True))

    # ------------------------------------------------------------ produce
    def produce(self, topic: str, values: Sequence, *, partition: int = 0, keys: Sequence | None = None,
                timestamps: Sequence[int] | None = None, headers: Sequence | None = None) -> int:
        """Appends one RecordBatch holding ``values`` to a partition; returns its base offset."""
        n = len(values)
        if n == 0:
            raise ValueError("nothing to produce")
        values = [_to_bytes(v) for v in values]
        keys = [None] * n if keys is None else [_to_bytes(k) for k in keys]
        now = int(time.time() * 1000)
        timestamps = [now] * n if timestamps is None else [int(t) for t in timestamps]
        headers = [None] * n if headers is None else [None if h is None else [(k, _to_bytes(v)) for k, v in h]
                                                      for h in headers]
        return self._b.append(self.pidx(topic, partition), values, keys, timestamps, headers)

    def fill(self, topic: str, n_per_partition: int, kind: str = "fixed_f32", *, size: int = 256,
             max_size: int | None = None, partitions: Iterable[int] | None = None, records_per_batch: int = 64,
             seed: int = 0, threads: int | None = None, keyed: bool = False) -> None:
        """Appends ``n_per_partition`` deterministic synthetic records to each partition.

        kinds: ``fixed_f32`` (``size`` floats: v[0]=offset, v[1]=partition), ``json_f32`` (JSON arrays of
        ``size..max_size`` numbers), ``bytes`` (``size..max_size`` bytes), ``tokens_i32``, ``varlen_f32``.
        ``keyed``: every record carries an 8-byte big-endian key, ``offset % 1000`` (a label).
        """
        k = _KINDS[kind]
        _, n, first = self.topic(topic)
        parts = list(range(n)) if partitions is None else list(partitions)
        pidxs = [first + p for p in parts]
        threads = threads or min(len(pidxs), max(1, min(16, (os.cpu_count() or 4))))
        self._b.fill_synthetic(pidxs, int(n_per_partition), k, int(size),
                               int(max_size if max_size is not None else size), int(records_per_batch), int(seed),
                               int(threads), bool(keyed))

    def copy_compressed(self, src_topic: str, dst_topic: str, compression: str | None, *,
                        partitions: Iterable[int] | None = None, level: int = 0, start_record: int = 0,
                        max_records: int = -1, threads: int | None = None) -> dict:
        """Appends the batches of ``src_topic``'s partitions holding records ``[start_record,
        max_records)`` of each (``-1``: to the end) to the same partitions of ``dst_topic``, each
        batch compressed as a producer with ``compression_type`` = ``compression`` ("gzip", "lz4",
        "zstd"; None: copied as they are) writes it: what a Kafka cluster's topic holds.  Served
        over the wire protocol, a KafkaBridge inflates them.  Returns ``{"raw_bytes",
        "compressed_bytes", "batches"}``."""
        codec = {None: 0, "none": 0, "gzip": 1, "lz4": 3, "zstd": 4}[compression]
        _, n, first = self.topic(src_topic)
        parts = list(range(n)) if partitions is None else list(partitions)
        dst = [self.pidx(dst_topic, p) for p in parts]
        threads = threads or min(len(parts), max(1, min(16, (os.cpu_count() or 4))))
        return dict(self._b.copy_compressed([first + p for p in parts], dst, codec, int(level), int(max_records),
                                            int(threads), int(start_record)))

    def delete_records(self, topic: str, partition: int, before_offset: int) -> None:
        self._b.delete_records(self.pidx(topic, partition), int(before_offset))

    # ------------------------------------------------------------ fault injection
    def inject_commit_failures(self, group: str, n: int = 1) -> None:
        self._b.inject_commit_failures(self._b.group_index(group, True), int(n))

    def set_fetch_delay(self, topic: str, partition: int, seconds: float) -> None:
        self._b.set_fetch_delay(self.pidx(topic, partition), int(seconds * 1e9))

    def inject_fetch_errors(self, topic: str, partition: int, n: int = 1) -> None:
        self._b.inject_fetch_errors(self.pidx(topic, partition), int(n))

    def partition_stats(self, topic: str, partition: int) -> dict:
        return self._b.partition_stats(self.pidx(topic, partition))


def _to_bytes(v):
    if v is None:
        return None
    if isinstance(v, str):
        return v.encode()
    if isinstance(v, (bytes, bytearray, memoryview)):
        return bytes(v)
    raise TypeError(f"record keys/values must be bytes or str, got {type(v).__name__}")


def open_broker(url: str) -> SyntheticBroker:
    """Per-process cached handle on an existing broker."""
    key = (os.getpid(), url)
    with _cache_lock:
        b = _cache.get(key)
        if b is None:
            b = SyntheticBroker(url, create=False)
            _cache[key] = b
        return b
