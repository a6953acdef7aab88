"""KafkaProducer over the synthetic broker (kafka-python compatible subset).

The reference only consumes; a producer is still part of what a user needs to
feed a topic (tests, benchmarks, examples).  Records are accumulated per
partition into RecordBatches of up to ``batch_size`` bytes and appended on
``flush()``, ``close()``, ``future.get()`` or when a batch fills up -- the
same batching a real producer does before a Produce request.  The default
partitioner is Kafka's: murmur2(key) for keyed records, round-robin otherwise.
"""
from __future__ import annotations

import copy
import functools
import itertools
import threading
import time

from ..broker.synthetic import open_broker, resolve_url
from .errors import KafkaConfigurationError
from .records import RecordMetadata, TopicPartition


def murmur2(data: bytes) -> int:
    """Kafka's murmur2 (the Java client's / kafka-python's DefaultPartitioner hash)."""
    length = len(data)
    seed = 0x9747B28C
    m = 0x5BD1E995
    r = 24
    h = seed ^ length
    length4 = length // 4
    for i in range(length4):
        i4 = i * 4
        k = ((data[i4] & 0xFF) + ((data[i4 + 1] & 0xFF) << 8) + ((data[i4 + 2] & 0xFF) << 16)
             + ((data[i4 + 3] & 0xFF) << 24))
        k = (k * m) & 0xFFFFFFFF
        k ^= (k % 0x100000000) >> r
        k = (k * m) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF
        h ^= k
    extra = length % 4
    if extra >= 3:
        h ^= (data[(length & ~3) + 2] & 0xFF) << 16
    if extra >= 2:
        h ^= (data[(length & ~3) + 1] & 0xFF) << 8
    if extra >= 1:
        h ^= data[length & ~3] & 0xFF
        h = (h * m) & 0xFFFFFFFF
    h ^= (h % 0x100000000) >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= (h % 0x100000000) >> 15
    return h


def default_partition(key: bytes | None, n_partitions: int, counter) -> int:
    if key is None:
        return next(counter) % n_partitions
    return (murmur2(key) & 0x7FFFFFFF) % n_partitions


class FutureRecordMetadata:
    """kafka-python's send() future: ``get``, ``is_done``, ``succeeded()``/``failed()``, ``value``/``exception``
    and ``add_callback``/``add_errback`` (run at flush time, or at once when already resolved)."""

    def __init__(self, producer: "KafkaProducer", tp: TopicPartition, idx: int, ts: int, ksize: int, vsize: int):
        self._producer, self._tp, self._idx, self._ts = producer, tp, idx, ts
        self._ksize, self._vsize = ksize, vsize
        self._offset = None
        self.exception = None
        self._callbacks: list = []
        self._errbacks: list = []

    def _metadata(self) -> RecordMetadata:
        return RecordMetadata(self._tp.topic, self._tp.partition, self._tp, self._offset, self._ts, None,
                              self._ksize, self._vsize, -1)

    def _resolve(self, base: int) -> None:
        self._offset = base + self._idx
        md = self._metadata()
        for f in self._callbacks:
            f(md)

    def _fail(self, exc: BaseException) -> None:
        self.exception = exc
        for f in self._errbacks:
            f(exc)

    @property
    def is_done(self) -> bool:
        return self._offset is not None or self.exception is not None

    @property
    def value(self):
        return self._metadata() if self._offset is not None else None

    def succeeded(self) -> bool:
        return self._offset is not None

    def failed(self) -> bool:
        return self.exception is not None

    def add_callback(self, fn, *args, **kwargs) -> "FutureRecordMetadata":
        f = functools.partial(fn, *args, **kwargs)
        if self._offset is not None:
            f(self._metadata())
        else:
            self._callbacks.append(f)
        return self

    def add_errback(self, fn, *args, **kwargs) -> "FutureRecordMetadata":
        f = functools.partial(fn, *args, **kwargs)
        if self.exception is not None:
            f(self.exception)
        else:
            self._errbacks.append(f)
        return self

    def get(self, timeout=None) -> RecordMetadata:
        if not self.is_done:
            self._producer.flush()
        if self.exception is not None:
            raise self.exception
        return self._metadata()


class KafkaProducer:
    DEFAULT_CONFIG = {
        "bootstrap_servers": "localhost",
        "client_id": None,
        "key_serializer": None,
        "value_serializer": None,
        "acks": 1,
        "compression_type": None,
        "retries": 0,
        "batch_size": 16384,
        "linger_ms": 0,
        "partitioner": None,
        "buffer_memory": 33554432,
        "max_block_ms": 60000,
        "max_request_size": 1048576,
        "request_timeout_ms": 30000,
        "api_version": None,
    }

    def __init__(self, **configs):
        extra = set(configs).difference(self.DEFAULT_CONFIG)
        if extra:
            raise KafkaConfigurationError(f"Unrecognized configs: {extra}")
        self.config = copy.copy(self.DEFAULT_CONFIG)
        self.config.update(configs)
        if self.config["compression_type"] not in (None, "none"):
            raise KafkaConfigurationError("the synthetic broker stores uncompressed batches only")
        self._broker = open_broker(resolve_url(self.config["bootstrap_servers"]))
        self._pending: dict[TopicPartition, list] = {}
        self._pending_bytes: dict[TopicPartition, int] = {}
        self._lock = threading.Lock()
        self._rr = itertools.count()
        self._closed = False

    def partitions_for(self, topic: str) -> set:
        return self._broker.partitions_for(topic)

    def send(self, topic: str, value=None, key=None, headers=None, partition=None, timestamp_ms=None):
        if self._closed:
            raise KafkaConfigurationError("producer is closed")
        if value is None and key is None:
            raise AssertionError("Need at least one: key or value")
        ks, vs = self.config["key_serializer"], self.config["value_serializer"]
        kb = ks(key) if ks is not None and key is not None else key
        vb = vs(value) if vs is not None and value is not None else value
        if isinstance(kb, str) or isinstance(vb, str):
            raise TypeError("keys and values must be bytes (configure a serializer)")
        n = self._broker.topic(topic)[1]
        if partition is None:
            part_fn = self.config["partitioner"]
            partition = part_fn(kb, list(range(n)), list(range(n))) if part_fn else default_partition(kb, n, self._rr)
        tp = TopicPartition(topic, int(partition))
        ts = int(time.time() * 1000) if timestamp_ms is None else int(timestamp_ms)
        size = (len(vb) if vb else 0) + (len(kb) if kb else 0) + 16
        with self._lock:
            lst = self._pending.setdefault(tp, [])
            fut = FutureRecordMetadata(self, tp, len(lst), ts, len(kb) if kb is not None else -1,
                                       len(vb) if vb is not None else -1)
            lst.append((vb, kb, ts, headers, fut))
            self._pending_bytes[tp] = self._pending_bytes.get(tp, 0) + size
            full = self._pending_bytes[tp] >= self.config["batch_size"]
        if full:
            self._flush_tp(tp)
        return fut

    def _flush_tp(self, tp: TopicPartition) -> None:
        with self._lock:
            recs = self._pending.pop(tp, [])
            self._pending_bytes.pop(tp, None)
        if not recs:
            return
        try:
            base = self._broker.produce(tp.topic, [r[0] for r in recs], partition=tp.partition,
                                        keys=[r[1] for r in recs], timestamps=[r[2] for r in recs],
                                        headers=[r[3] for r in recs])
        except Exception as exc:  # noqa: BLE001 - handed to the futures, as kafka-python does
            for r in recs:
                r[4]._fail(exc)
            return
        for r in recs:
            r[4]._resolve(base)

    def flush(self, timeout=None) -> None:
        for tp in list(self._pending):
            self._flush_tp(tp)

    def close(self, timeout=None) -> None:
        if not self._closed:
            self.flush()
            self._closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
