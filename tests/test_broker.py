"""Synthetic broker: log store, offsets, groups, persistence, multi-process safety, fault injection."""
import multiprocessing as mp
import os
import shutil
import tempfile
import time

import pytest

from torchkafka_amd.broker import SyntheticBroker, open_broker, resolve_url
from torchkafka_amd.client.errors import CommitFailedError, KafkaError, NoBrokersAvailable
from torchkafka_amd.client.records import TopicPartition
from torchkafka_amd.ops.native import core


def test_topics_and_offsets(broker):
    broker.create_topic("a", 3)
    broker.create_topic("a", 3)  # idempotent
    broker.create_topic("b", 1)
    assert broker.topics() == ["a", "b"]
    assert broker.partitions_for("a") == {0, 1, 2}
    assert broker.end_offsets("a") == {0: 0, 1: 0, 2: 0}
    assert broker.produce("a", [b"x", b"y"], partition=1) == 0
    assert broker.produce("a", [b"z"], partition=1) == 2
    assert broker.end_offset("a", 1) == 3
    with pytest.raises(KafkaError):
        broker.topic("missing")
    with pytest.raises(KafkaError):
        broker.pidx("a", 3)


def test_no_broker():
    with pytest.raises(NoBrokersAvailable):
        SyntheticBroker("shm://does-not-exist-xyz")
    os.environ.pop("TORCHKAFKA_BROKER", None)
    with pytest.raises(NoBrokersAvailable):
        resolve_url("localhost:9092")
    os.environ["TORCHKAFKA_BROKER"] = "shm://somewhere"
    try:
        assert resolve_url(["localhost:9092"]) == "shm://somewhere"
    finally:
        del os.environ["TORCHKAFKA_BROKER"]


def test_fill_synthetic_and_fetch_bytes(broker):
    broker.create_topic("t", 4)
    broker.fill("t", 1000, "fixed_f32", size=256, records_per_batch=100)
    assert broker.end_offsets("t") == {p: 1000 for p in range(4)}
    st = broker.partition_stats("t", 0)
    assert st["batches"] == 10 and st["records_produced"] == 1000
    assert st["log_bytes"] > 1000 * 1024


def test_log_full_raises(broker):
    broker.create_topic("small", 1, log_capacity=4096)
    with pytest.raises(KafkaError, match="full"):
        broker.produce("small", [b"x" * 5000])


def test_committed_offsets_persist_across_reopen():
    d = tempfile.mkdtemp(prefix="tkbroker-")
    url = f"file://{d}/broker"
    try:
        b = SyntheticBroker.create(url)
        b.create_topic("t", 2)
        b.produce("t", [b"a", b"b", b"c"], partition=1)
        b.commit("grp", {TopicPartition("t", 1): 2})
        del b
        b2 = SyntheticBroker(url)  # a "restart": new handle on the same directory
        assert b2.committed("grp", "t", 1) == 2
        assert b2.committed("grp", "t", 0) is None
        assert b2.end_offset("t", 1) == 3
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _producer_proc(url, part, n):
    b = SyntheticBroker(url)
    for i in range(n):
        b.produce("t", [f"{part}-{i}".encode()], partition=part)


def test_multiprocess_producers(broker):
    broker.create_topic("t", 2)
    ctx = mp.get_context("fork")
    procs = [ctx.Process(target=_producer_proc, args=(broker.url, i % 2, 200)) for i in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert broker.end_offsets("t") == {0: 400, 1: 400}
    recs = []
    from torchkafka_amd.client import KafkaConsumer

    c = KafkaConsumer("t", bootstrap_servers=broker.url, auto_offset_reset="earliest", consumer_timeout_ms=100)
    recs = [(r.partition, r.offset) for r in c]
    assert sorted(recs) == [(p, o) for p in range(2) for o in range(400)]


def test_group_range_assignment_and_rebalance(broker):
    b = broker.native
    broker.create_topic("t", 5)
    ti = broker.topic("t")[0]
    g = b.group_index("grp")
    s1 = b.join_group(g, [ti], 10000, 300000)
    m1 = b.member_id(g, s1)
    time.sleep(0.35)  # initial rebalance delay (300 ms in the fixture)
    gen1, state, active, asg = b.poll_group(g, s1, m1)
    assert active and state == 2 and asg == [0, 1, 2, 3, 4]
    s2 = b.join_group(g, [ti], 10000, 300000)
    m2 = b.member_id(g, s2)
    # Kafka's PreparingRebalance: the first member must rejoin before anything is reassigned, and
    # may still commit with its current generation until it does
    g_prep, st_prep, active, asg_prep = b.poll_group(g, s1, m1)
    assert (g_prep, st_prep, active, asg_prep) == (gen1, 1, True, [])
    b.commit(g, s1, m1, gen1, [(4, 3, "")])
    assert b.committed(g, 4) == (3, "")
    b.rejoin_group(g, s1, m1)
    gen2, _, _, asg1 = b.poll_group(g, s1, m1)
    _, _, _, asg2 = b.poll_group(g, s2, m2)
    assert gen2 == gen1 + 1
    assert asg1 == [0, 1, 2] and asg2 == [3, 4]  # range assignor: first member gets the extra partition
    # a commit with the old generation fails like Kafka's ILLEGAL_GENERATION
    with pytest.raises(CommitFailedError):
        b.commit(g, s1, m1, gen1, [(0, 1, "")])
    b.commit(g, s1, m1, gen2, [(0, 1, "meta")])
    assert b.committed(g, 0) == (1, "meta")
    # a non-member commit is rejected while the group has members
    with pytest.raises(CommitFailedError):
        b.commit(g, -1, 0, 0, [(0, 2, "")])
    b.leave_group(g, s2, m2)  # a member leaves: the one left rejoins, then takes everything
    assert b.poll_group(g, s1, m1)[1] == 1
    b.rejoin_group(g, s1, m1)
    gen3, _, _, asg1 = b.poll_group(g, s1, m1)
    assert gen3 == gen2 + 1 and asg1 == [0, 1, 2, 3, 4]


def _join_and_die(url, ti):
    b = SyntheticBroker(url).native
    g = b.group_index("grp")
    b.join_group(g, [ti], 10000, 300000)
    os._exit(0)  # dies without leaving the group


def test_dead_member_is_evicted(broker):
    b = broker.native
    broker.create_topic("t", 2)
    ti = broker.topic("t")[0]
    p = mp.get_context("fork").Process(target=_join_and_die, args=(broker.url, ti))
    p.start()
    p.join(10)
    g = b.group_index("grp")
    s = b.join_group(g, [ti], 10000, 300000)
    m = b.member_id(g, s)
    deadline = time.time() + 2
    while time.time() < deadline:
        _, state, _, asg = b.poll_group(g, s, m)
        if state == 2 and asg == [0, 1]:
            break
        time.sleep(0.02)
    assert asg == [0, 1]


def test_max_poll_interval_eviction(broker):
    b = broker.native
    broker.create_topic("t", 1)
    ti = broker.topic("t")[0]
    g = b.group_index("slow")
    s = b.join_group(g, [ti], 10000, 50)  # 50 ms max poll interval
    m = b.member_id(g, s)
    gen, state, active, _ = b.poll_group(g, s, m)  # polled in time
    time.sleep(0.12)
    with pytest.raises(CommitFailedError, match="max_poll_interval"):
        b.commit(g, s, m, gen, [(broker.pidx("t", 0), 0, "")])


def test_commit_failure_injection(broker):
    broker.create_topic("t", 1)
    broker.inject_commit_failures("g", 2)
    tp = TopicPartition("t", 0)
    for _ in range(2):
        with pytest.raises(CommitFailedError):
            broker.commit("g", {tp: 1})
    broker.commit("g", {tp: 1})
    assert broker.committed("g", "t", 0) == 1


def test_open_broker_cache_is_per_process(broker):
    assert open_broker(broker.url) is open_broker(broker.url)


def test_crc_hw_path_reported():
    assert isinstance(core().crc32c_hw(), bool)
