"""DeviceLoader commit sinks and the `_process` contract (CPU).

* commit_sink='worker': the offsets the user finished are published to the worker that delivered
  each partition and committed by that worker's own consumer -- as a group member with its
  generation under sharding='group' (a commit from outside the group would be rejected), through
  kafka-python when that is the consumer.  With the reference's multi-worker messages
  (kafka_dataset.py:127, 140-143).
* A dataset that declares a schema AND overrides `_process` is served by the reference's
  per-record loop (kafka_dataset.py:156-162): its filter applies, and the skipped records are
  committed with the next commit (B6).
* kafka-python is not installed here: a test double injected as the `kafka` module stands in for
  it (parity with the real library stays unpinned).
"""
import json
import logging
import os
import sys
import types
from collections import namedtuple

import torch

from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit


class Vec8(KafkaDataset):
    schema = FixedWidth(torch.float32, (8,))


def _loader(ds_cls, broker, bs, **kw):
    consumer_kw = {"consumer_timeout_ms": 500, **kw.pop("consumer_kw", {})}
    return DeviceLoader(ds_cls.placeholder(), bs, device="cpu", num_workers=kw.pop("workers", 2),
                        worker_init_fn=ds_cls.init_worker("t", bootstrap_servers=broker.url,
                                                          group_id=kw.pop("group", "g"),
                                                          auto_offset_reset="earliest", **consumer_kw), **kw)


def test_group_sharding_auto_commit_commits_as_members(broker):
    """ADVICE: with sharding='group' every worker is a group member, so the main process may not
    commit for them; the worker sink makes each member commit its own partitions."""
    broker.create_topic("t", 4)
    broker.fill("t", 30, "fixed_f32", size=8)
    dl = _loader(Vec8, broker, 10, sharding="group", consumer_kw={"consumer_timeout_ms": 700})
    assert dl._sink == "worker"
    n = sum(x.shape[0] for x in auto_commit(dl))
    assert n == 120
    assert broker.committed_offsets("g", "t") == {p: 30 for p in range(4)}


def test_worker_sink_on_static_sharding_matches_broker_sink(broker):
    broker.create_topic("t", 3)
    broker.fill("t", 40, "fixed_f32", size=8)
    for sink, group in (("broker", "gb"), ("worker", "gw")):
        dl = _loader(Vec8, broker, 16, group=group, commit_sink=sink)
        assert dl._sink == sink
        assert sum(x.shape[0] for x in auto_commit(dl)) == 120
        assert broker.committed_offsets(group, "t") == {0: 40, 1: 40, 2: 40}


def test_worker_sink_logs_like_reference_workers(broker, caplog):
    """Worker-side commits log 'Committing offsets on worker %d.' (INFO) as the reference's
    workers do; captured here through the commits' effect and the main-process silence."""
    broker.create_topic("t", 1)
    broker.fill("t", 20, "fixed_f32", size=8)
    with caplog.at_level(logging.DEBUG, logger="torchkafka.kafka_dataset"):
        list(auto_commit(_loader(Vec8, broker, 10, workers=1, commit_sink="worker")))
    # the commit messages are emitted in the worker process; the main process stores nothing itself
    assert not [r for r in caplog.records if r.getMessage() == "Committed offsets."]
    assert broker.committed_offsets("g", "t") == {0: 20}


class EvenOnly(KafkaDataset):
    schema = FixedWidth(torch.float32, (8,))

    def _process(self, record):
        if record.offset % 2:
            return None  # the reference's None-skip (B6)
        return self.schema.process(record) * 2


def test_overridden_process_is_honoured_with_a_schema(broker):
    broker.create_topic("t", 2)
    broker.fill("t", 30, "fixed_f32", size=8)
    dl = _loader(EvenOnly, broker, 5)
    assert dl.plan.process_overridden and not dl.plan.fast_path
    xs = torch.cat(list(auto_commit(dl)))
    offsets = sorted((xs[:, 0] / 2).long().tolist())
    assert len(offsets) == 30 and all(o % 2 == 0 for o in offsets)
    assert torch.equal(xs[:, 1] / 2, (xs[:, 1] / 2).round())  # the transform ran (x2)
    # skipped odd offsets are committed with their batch: everything consumed is committed
    assert broker.committed_offsets("g", "t") == {0: 30, 1: 30}


# ------------------------------------------------------------------ kafka-python test double
_TP = namedtuple("TopicPartition", ["topic", "partition"])
_OAM = namedtuple("OffsetAndMetadata", ["offset", "metadata"])
_CR = namedtuple("ConsumerRecord", ["topic", "partition", "offset", "timestamp", "timestamp_type", "key", "value",
                                    "headers", "checksum", "serialized_key_size", "serialized_value_size",
                                    "serialized_header_size"])


def _fake_kafka_module(log_path: str, n_parts: int, per_part: int):
    import struct

    class CommitFailedError(Exception):
        pass

    class KafkaConsumer:
        """Just enough of kafka-python 2.0.2: subscribe, poll, commit(offsets), close.  Group
        assignment is simulated: DataLoader worker w of n takes partitions p % n == w."""

        def __init__(self, *topics, **config):
            from torch.utils.data import get_worker_info

            self.config = {"consumer_timeout_ms": float("inf"), **config}
            assert config.get("enable_auto_commit") is False  # B1
            self._topics = set(topics)
            wi = get_worker_info()
            w, n = (wi.id, wi.num_workers) if wi is not None else (0, 1)
            self._pos = {_TP(t, p): 0 for t in sorted(topics) for p in range(n_parts) if p % n == w}
            self._w = w

        def subscription(self):
            return set(self._topics)

        def poll(self, timeout_ms=0, max_records=None):
            out, left = {}, max_records or 500
            for tp, pos in self._pos.items():
                if left <= 0:
                    break
                take = min(left, per_part - pos)
                if take > 0:
                    out[tp] = [_CR(tp.topic, tp.partition, o, 0, 0, None,
                                   struct.pack("<8f", float(o), float(tp.partition), *([0.5] * 6)), [], None, -1,
                                   32, -1) for o in range(pos, pos + take)]
                    self._pos[tp] = pos + take
                    left -= take
            return out

        def commit(self, offsets=None):
            with open(log_path, "a") as f:
                for tp, om in offsets.items():
                    f.write(json.dumps({"worker": self._w, "topic": tp.topic, "partition": tp.partition,
                                        "offset": om.offset}) + "\n")

        def close(self, autocommit=True):
            pass

    kafka = types.ModuleType("kafka")
    kafka.KafkaConsumer = KafkaConsumer
    errors = types.ModuleType("kafka.errors")
    errors.CommitFailedError = CommitFailedError
    structs = types.ModuleType("kafka.structs")
    structs.TopicPartition, structs.OffsetAndMetadata = _TP, _OAM
    kafka.errors, kafka.structs = errors, structs
    return {"kafka": kafka, "kafka.errors": errors, "kafka.structs": structs}


def test_kafka_python_consumer_commits_through_its_worker(tmp_path, monkeypatch):
    log_path = str(tmp_path / "commits.jsonl")
    for name, mod in _fake_kafka_module(log_path, n_parts=3, per_part=25).items():
        monkeypatch.setitem(sys.modules, name, mod)
    monkeypatch.delenv("TORCHKAFKA_BROKER", raising=False)
    dl = DeviceLoader(Vec8.placeholder(), 10, device="cpu", num_workers=2, sharding="group",
                      worker_init_fn=Vec8.init_worker("t", bootstrap_servers="kafka-1:9092", group_id="g",
                                                      consumer_timeout_ms=300))
    assert dl._sink == "worker" and not dl.plan.span
    xs = torch.cat(list(auto_commit(dl)))
    assert sorted(map(tuple, xs[:, :2].long().tolist())) == sorted((o, p) for p in range(3) for o in range(25))
    final = {}
    for line in open(log_path):
        c = json.loads(line)
        assert c["worker"] == c["partition"] % 2  # each partition committed by its own consumer
        final[c["partition"]] = max(final.get(c["partition"], 0), c["offset"])
    assert final == {0: 25, 1: 25, 2: 25}
    assert os.path.getsize(log_path) > 0
