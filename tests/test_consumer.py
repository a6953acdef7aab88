"""KafkaConsumer / KafkaProducer: kafka-python compatible behaviour over the synthetic broker."""
import json
import time

import pytest

from torchkafka_amd.client import KafkaConsumer, KafkaProducer, OffsetAndMetadata, TopicPartition
from torchkafka_amd.client.errors import (
    CommitFailedError, IllegalStateError, KafkaConfigurationError, NoOffsetForPartitionError,
)
from torchkafka_amd.client.producer import murmur2


def consumer(broker, *topics, **kw):
    kw.setdefault("bootstrap_servers", broker.url)
    kw.setdefault("auto_offset_reset", "earliest")
    kw.setdefault("consumer_timeout_ms", 100)
    return KafkaConsumer(*topics, **kw)


def test_unknown_config_rejected(broker):
    with pytest.raises(KafkaConfigurationError):
        KafkaConsumer(bootstrap_servers=broker.url, not_a_config=1)


def test_iteration_offsets_keys_headers(broker):
    broker.create_topic("t", 1)
    broker.produce("t", [b"v0", b"v1", None], keys=[b"k", None, b"k2"], timestamps=[10, 20, 30],
                   headers=[[("h", b"1")], None, None])
    c = consumer(broker, "t", group_id="g")
    recs = list(c)
    assert [r.offset for r in recs] == [0, 1, 2]
    assert [r.value for r in recs] == [b"v0", b"v1", None]
    assert [r.key for r in recs] == [b"k", None, b"k2"]
    assert recs[0].headers == [("h", b"1")] and recs[1].headers == []
    assert [r.timestamp for r in recs] == [10, 20, 30]
    assert recs[0].topic == "t" and recs[0].partition == 0 and recs[0].timestamp_type == 0
    assert recs[0].serialized_value_size == 2 and recs[2].serialized_value_size == -1


def test_deserializers(broker):
    broker.create_topic("t", 1)
    broker.produce("t", [json.dumps([1, 2]).encode()], keys=[b"key"])
    c = consumer(broker, "t", value_deserializer=json.loads, key_deserializer=bytes.decode)
    r = next(iter(c))
    assert r.value == [1, 2] and r.key == "key"


def test_consumer_timeout_stops_iteration(broker):
    broker.create_topic("t", 1)
    c = consumer(broker, "t", consumer_timeout_ms=50)
    t0 = time.monotonic()
    assert list(c) == []
    assert 0.04 < time.monotonic() - t0 < 2.0


def test_auto_offset_reset_latest_and_none(broker):
    broker.create_topic("t", 1)
    broker.produce("t", [b"old"])
    c = consumer(broker, "t", auto_offset_reset="latest")
    assert list(c) == []
    c2 = consumer(broker, auto_offset_reset="none", group_id="g")
    with pytest.raises(NoOffsetForPartitionError):
        c2.assign([TopicPartition("t", 0)])


def test_commit_and_resume_from_committed(broker):
    broker.create_topic("t", 2)
    for p in range(2):
        broker.produce("t", [f"{p}-{i}".encode() for i in range(10)], partition=p)
    c = consumer(broker, "t", group_id="g", enable_auto_commit=False)
    got = [next(c) for _ in range(7)]
    c.commit()
    # committed = consumed positions only (records still buffered are not committed)
    committed = {p: broker.committed("g", "t", p) for p in range(2)}
    consumed = {0: 0, 1: 0}  # kafka-python commits every assigned partition's consumed position
    for r in got:
        consumed[r.partition] = r.offset + 1
    assert committed == consumed
    c.close()
    c2 = consumer(broker, "t", group_id="g", enable_auto_commit=False)
    rest = list(c2)
    assert len(rest) == 20 - 7
    assert not ({(r.partition, r.offset) for r in rest} & {(r.partition, r.offset) for r in got})


def test_commit_requires_group_id(broker):
    broker.create_topic("t", 1)
    c = consumer(broker, "t")
    with pytest.raises(AssertionError):
        c.commit()


def test_commit_explicit_offsets_and_metadata(broker):
    broker.create_topic("t", 1)
    broker.produce("t", [b"a", b"b"])
    c = consumer(broker, group_id="g")
    tp = TopicPartition("t", 0)
    c.assign([tp])
    c.commit({tp: OffsetAndMetadata(1, "m")})
    assert c.committed(tp) == 1
    assert c.committed(tp, metadata=True) == OffsetAndMetadata(1, "m")


def test_poll_returns_dict_by_partition(broker):
    broker.create_topic("t", 3)
    for p in range(3):
        broker.produce("t", [b"x"] * 4, partition=p)
    c = consumer(broker, "t")
    out = {}
    deadline = time.time() + 2
    while sum(len(v) for v in out.values()) < 12 and time.time() < deadline:
        for tp, recs in c.poll(timeout_ms=50, max_records=5).items():
            out.setdefault(tp, []).extend(recs)
    assert {tp.partition for tp in out} == {0, 1, 2}
    assert all(len(v) == 4 for v in out.values())


def test_seek_position_pause(broker):
    broker.create_topic("t", 2)
    for p in range(2):
        broker.produce("t", [b"x"] * 5, partition=p)
    c = consumer(broker)
    tp0, tp1 = TopicPartition("t", 0), TopicPartition("t", 1)
    c.assign([tp0, tp1])
    assert c.assignment() == {tp0, tp1}
    c.seek(tp0, 3)
    assert c.position(tp0) == 3
    c.pause(tp1)
    recs = list(c)
    assert {(r.partition, r.offset) for r in recs} == {(0, 3), (0, 4)}
    c.resume(tp1)
    c.seek_to_beginning(tp1)
    assert len(list(c)) == 5
    assert c.end_offsets([tp0]) == {tp0: 5} and c.beginning_offsets([tp0]) == {tp0: 0}
    assert c.partitions_for_topic("t") == {0, 1} and "t" in c.topics()


def test_subscribe_assign_exclusive(broker):
    broker.create_topic("t", 1)
    c = consumer(broker, "t")
    with pytest.raises(IllegalStateError):
        c.assign([TopicPartition("t", 0)])


def test_group_members_split_partitions(broker):
    broker.create_topic("t", 4)
    for p in range(4):
        broker.produce("t", [b"x"] * 3, partition=p)
    c1 = consumer(broker, "t", group_id="g", consumer_timeout_ms=300)
    c2 = consumer(broker, "t", group_id="g", consumer_timeout_ms=300)
    c1.assignment(), c2.assignment()  # both join inside the initial rebalance delay
    time.sleep(0.35)
    a1, a2 = c1.assignment(), c2.assignment()
    assert a1 | a2 == {TopicPartition("t", p) for p in range(4)} and not (a1 & a2)
    assert len(a1) == len(a2) == 2


def test_stale_generation_commit_fails(broker):
    """Kafka's rebalance round: a joining member waits for the others to rejoin; until c1 does, its
    current-generation commit is accepted; once the round completed without it (its rebalance
    timeout, max_poll_interval_ms, expired) its commit is rejected and it rejoins as a new member."""
    import threading

    broker.create_topic("t", 2)
    c1 = consumer(broker, "t", group_id="g", enable_auto_commit=False, max_poll_interval_ms=400)
    c1.assignment()
    time.sleep(0.35)
    assert len(c1.assignment()) == 2
    c2 = consumer(broker, "t", group_id="g")
    done = threading.Event()
    th = threading.Thread(target=lambda: (c2.assignment(), done.set()))
    th.start()  # joins: blocks until every member rejoined (or c1's rebalance timeout)
    time.sleep(0.05)
    assert not done.is_set()
    c1.commit()  # the group is preparing a rebalance: c1's generation is still current
    th.join(timeout=10)  # c1 never rejoined: dropped at its rebalance timeout, c2 gets everything
    assert done.is_set() and len(c2.assignment()) == 2
    with pytest.raises(CommitFailedError):
        c1.commit()


def test_max_poll_interval_exceeded(broker):
    broker.create_topic("t", 1)
    broker.produce("t", [b"x"])
    c = consumer(broker, "t", group_id="g", max_poll_interval_ms=50, consumer_timeout_ms=300)
    next(c)
    time.sleep(0.15)
    with pytest.raises(CommitFailedError):
        c.commit()


def test_forked_consumer_detected(broker):
    import multiprocessing as mp

    broker.create_topic("t", 1)
    c = consumer(broker, "t")

    def child(q):
        try:
            next(c)
            q.put("no error")
        except IllegalStateError as e:
            q.put(str(e))

    q = mp.get_context("fork").Queue()
    p = mp.get_context("fork").Process(target=child, args=(q,))
    p.start()
    msg = q.get(timeout=10)
    p.join(10)
    assert "placeholder()" in msg


def test_close_is_idempotent_and_blocks_use(broker):
    broker.create_topic("t", 1)
    c = consumer(broker, "t")
    c.close(autocommit=False)
    c.close()
    with pytest.raises(IllegalStateError):
        next(c)


def test_murmur2_matches_kafka():
    # vectors from Kafka's Java client (UtilsTest) / kafka-python tests
    def signed(h):
        return h - (1 << 32) if h & 0x80000000 else h

    assert signed(murmur2(b"21")) == -973932308
    assert signed(murmur2(b"foobar")) == -790332482
    assert signed(murmur2(b"a-little-bit-long-string")) == -985981536
    assert signed(murmur2(b"a-little-bit-longer-string")) == -1486304829
    assert signed(murmur2(b"lkjh234lh9fiuh90y23oiuhsafujhadof229phr9h19h89h8")) == -58897971
    assert signed(murmur2(b"abc")) == 479470107


def test_producer_partitioning_and_futures(broker):
    broker.create_topic("t", 4)
    p = KafkaProducer(bootstrap_servers=broker.url, value_serializer=lambda v: json.dumps(v).encode())
    futs = [p.send("t", {"i": i}, key=f"user-{i % 3}".encode()) for i in range(30)]
    md = [f.get() for f in futs]
    by_key = {}
    for i, m in enumerate(md):
        by_key.setdefault(i % 3, set()).add(m.partition)
    assert all(len(s) == 1 for s in by_key.values())  # same key -> same partition
    rr = [p.send("t", {"i": i}).get().partition for i in range(8)]
    assert set(rr) == {0, 1, 2, 3}
    p.close()
    assert sum(broker.end_offsets("t").values()) == 38


def test_poll_without_update_offsets_peeks(broker):
    broker.create_topic("t", 1)
    broker.produce("t", [b"a", b"b", b"c"], partition=0)
    c = consumer(broker, "t")
    tp = TopicPartition("t", 0)
    peek = {}
    deadline = time.time() + 2
    while not peek and time.time() < deadline:
        peek = c.poll(timeout_ms=50, max_records=2, update_offsets=False)
    assert [r.offset for r in peek[tp]] == [0, 1]
    assert c.position(tp) == 0
    got = c.poll(timeout_ms=500, max_records=2)
    assert [r.offset for r in got[tp]] == [0, 1]
    assert c.position(tp) == 2


def test_offsets_for_times(broker):
    broker.create_topic("t", 2)
    broker.produce("t", [b"a", b"b", b"c"], partition=0, timestamps=[100, 200, 300])
    broker.produce("t", [b"d", b"e"], partition=0, timestamps=[250, 400])
    broker.produce("t", [b"x"], partition=1, timestamps=[50])
    c = consumer(broker, "t")
    tp0, tp1 = TopicPartition("t", 0), TopicPartition("t", 1)
    got = c.offsets_for_times({tp0: 150, tp1: 10})
    assert (got[tp0].offset, got[tp0].timestamp) == (1, 200)
    assert (got[tp1].offset, got[tp1].timestamp) == (0, 50)
    # first record at or after the time, not the first batch whose max covers it
    assert c.offsets_for_times({tp0: 240})[tp0] == (2, 300)
    assert c.offsets_for_times({tp0: 350})[tp0] == (4, 400)
    assert c.offsets_for_times({tp0: 401, tp1: 51}) == {tp0: None, tp1: None}
    broker.delete_records("t", 0, 2)
    assert c.offsets_for_times({tp0: 0})[tp0] == (2, 300)
    with pytest.raises(ValueError):
        c.offsets_for_times({tp0: -1})


def test_producer_future_callbacks_and_errbacks(broker):
    broker.create_topic("t", 1)
    p = KafkaProducer(bootstrap_servers=broker.url)
    seen, errs = [], []
    fut = p.send("t", b"v0").add_callback(seen.append).add_errback(errs.append)
    assert not fut.is_done and not fut.succeeded() and fut.value is None
    p.flush()
    assert fut.is_done and fut.succeeded() and not fut.failed()
    assert [m.offset for m in seen] == [0] and fut.value.offset == 0 and not errs
    late = []
    fut.add_callback(lambda tag, md: late.append((tag, md.offset)), "x")  # already resolved: runs at once
    assert late == [("x", 0)]
    bad = p.send("t", b"v1", partition=7).add_errback(errs.append)  # no partition 7: fails at flush
    p.flush()
    assert bad.failed() and bad.is_done and len(errs) == 1 and bad.exception is errs[0]
    with pytest.raises(type(errs[0])):
        bad.get()
    p.close()


def test_commit_async_future(broker):
    broker.create_topic("t", 1)
    broker.produce("t", [b"a", b"b"], partition=0)
    c = consumer(broker, "t", group_id="ga")
    assert len(list(c)) == 2
    seen = []
    fut = c.commit_async(callback=lambda offs, exc: seen.append(exc))
    assert fut.is_done and fut.succeeded() and seen == [None]
    assert broker.committed("ga", "t", 0) == 2
    broker.inject_commit_failures("ga", 1)
    errs = []
    fut = c.commit_async().add_errback(errs.append)
    assert fut.failed() and isinstance(errs[0], CommitFailedError)
    with pytest.raises(CommitFailedError):
        fut.get()


def test_commit_async_callback_gets_committed_offsets(broker):
    broker.create_topic("t", 2)
    broker.produce("t", [b"a", b"b", b"c"], partition=0)
    broker.produce("t", [b"d"], partition=1)
    seen = []
    c = consumer(broker, "t", group_id="gb", default_offset_commit_callback=lambda o, e: seen.append((o, e)))
    assert len(list(c)) == 4
    fut = c.commit_async()  # no callback: kafka-python's default_offset_commit_callback runs
    want = {TopicPartition("t", 0): OffsetAndMetadata(3, ""), TopicPartition("t", 1): OffsetAndMetadata(1, "")}
    assert seen == [(want, None)] and fut.value == want
    got = []
    tp = TopicPartition("t", 0)
    c.commit_async({tp: 2}, callback=lambda o, e: got.append((o, e)))
    assert got == [({tp: OffsetAndMetadata(2, "")}, None)]
    assert broker.committed("gb", "t", 0) == 2
    broker.inject_commit_failures("gb", 1)
    fut = c.commit_async(callback=lambda o, e: got.append((o, e)))
    assert fut.failed() and isinstance(got[-1][1], CommitFailedError) and got[-1][0] == want
