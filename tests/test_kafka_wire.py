"""Kafka wire protocol: the native replicator (KafkaBridge) against a Kafka-protocol server (CPU).

The reference consumes a real cluster through kafka-python (/root/reference/src/kafka_dataset.py:
21-22, 206).  No cluster exists here, so `KafkaWireServer` serves a synthetic broker over the
Kafka protocol (ApiVersions, Metadata, ListOffsets, Fetch v4, FindCoordinator, OffsetCommit v2,
OffsetFetch v1) and the native replicator (csrc/core/replicator.cpp) mirrors it into a local
broker that the loader reads.  Parity with a real Kafka broker is unpinned (none is reachable);
the server follows the protocol's published request/response layouts.
"""
import os
import time
import uuid

import pytest
import torch

from conftest import synth_f32
from torchkafka_amd import DeviceLoader, FixedWidth, KafkaConsumer, KafkaDataset, auto_commit
from torchkafka_amd.broker import KafkaBridge, KafkaWireServer, SyntheticBroker
from torchkafka_amd.broker.wire_server import NOT_LEADER, control_batch
from torchkafka_amd.client.records import TopicPartition
from torchkafka_amd.ops.native import core


@pytest.fixture
def server(broker):
    srv = KafkaWireServer(broker).start()
    try:
        yield srv
    finally:
        srv.close()


def bridge(srv, topic="t", **kw):
    kw.setdefault("log_capacity", 64 << 20)
    kw.setdefault("index_capacity", 1 << 16)
    kw.setdefault("url", f"shm://tkbr-{os.getpid()}-{uuid.uuid4().hex[:8]}")
    b = KafkaBridge(srv.address, topic, **kw)
    b._own = True  # tests: remove the local replica on close
    return b


def wait_for(cond, timeout=10.0):
    t = time.monotonic() + timeout
    while time.monotonic() < t:
        if cond():
            return True
        time.sleep(0.005)
    return False


def log_bytes(b: SyntheticBroker, topic, p):
    pidx = b.pidx(topic, p)
    return b.native.read_log(pidx, 0, b.native.log_bytes(pidx))


def test_wire_client_metadata_offsets_and_commits(broker, server):
    broker.create_topic("t", 3)
    broker.fill("t", 100, "fixed_f32", size=8, records_per_batch=16)
    c = core().WireClient(server.address)
    err, parts = c.metadata("t")
    assert err == 0 and [p[0] for p in parts] == [0, 1, 2] and all(p[1] == 0 for p in parts)
    assert c.metadata("nope")[0] == 3  # UnknownTopicOrPartition
    assert c.list_offsets("t", [0, 1, 2], -1) == {0: 100, 1: 100, 2: 100}
    assert c.list_offsets("t", [1], -2) == {1: 0}
    assert c.offset_fetch("g", "t", [0, 1]) == {0: -1, 1: -1}
    assert c.offset_commit("g", "t", {0: 17, 2: 99}) == {0: 0, 2: 0}
    assert broker.committed_offsets("g", "t") == {0: 17, 1: None, 2: 99}
    assert c.offset_fetch("g", "t", [0, 2]) == {0: 17, 2: 99}
    assert core().WireClient.parse_bootstrap("kafka://h1:9093, h2") == [("h1", 9093), ("h2", 9092)]


def test_replica_logs_are_byte_identical(broker, server):
    broker.create_topic("t", 4)
    broker.fill("t", 700, "fixed_f32", size=32, records_per_batch=50)
    with bridge(server, group_id="g") as br:
        assert br.wait_caught_up(10)
        for p in range(4):
            assert br.local.end_offset("t", p) == 700
            assert log_bytes(br.local, "t", p) == log_bytes(broker, "t", p)
        st = br.stats()
        assert all(s["fetch_offset"] == 700 and s["batches"] == 14 for s in st)
        assert br.errors == 0


def test_live_stream_and_small_fetches(broker, server):
    """A record set cut at max_partition_fetch_bytes keeps only whole batches; the rest is refetched."""
    broker.create_topic("t", 2)
    broker.fill("t", 200, "fixed_f32", size=64, records_per_batch=20)  # ~5.5 KB batches
    with bridge(server, max_partition_fetch_bytes=8192, fetch_max_bytes=16384, fetch_max_wait_ms=5) as br:
        assert br.wait_caught_up(10)
        broker.fill("t", 300, "fixed_f32", size=64, records_per_batch=30)  # produced while mirroring
        assert br.wait_caught_up(10)
        for p in range(2):
            assert br.local.end_offset("t", p) == 500
            assert log_bytes(br.local, "t", p) == log_bytes(broker, "t", p)
        assert min(s["fetches"] for s in br.stats()) > 10


def test_partial_trailing_batches(broker, server):
    broker.create_topic("t", 1)
    broker.fill("t", 400, "fixed_f32", size=16, records_per_batch=40)
    server.partial_tail = True
    with bridge(server) as br:
        assert br.wait_caught_up(10)
        assert log_bytes(br.local, "t", 0) == log_bytes(broker, "t", 0)
        assert br.errors == 0


def test_starts_at_the_groups_committed_offset_or_reset(broker, server):
    broker.create_topic("t", 2)
    broker.fill("t", 100, "fixed_f32", size=8, records_per_batch=10)
    broker.commit("g", {TopicPartition("t", 0): 35})
    with bridge(server, group_id="g") as br:
        assert br.wait_caught_up(10)
        st = {s["partition"]: s for s in br.stats()}
        assert st[0]["start_offset"] == 35 and st[1]["start_offset"] == 0
        assert br.local.committed("g", "t", 0) == 35  # seeded for the local consumers
        c = KafkaConsumer("t", bootstrap_servers=br.url, group_id="g", auto_offset_reset="earliest",
                          enable_auto_commit=False, consumer_timeout_ms=300)
        offs = {0: [], 1: []}
        for r in c:
            offs[r.partition].append(r.offset)
        c.close()
        assert offs[0] == list(range(35, 100)) and offs[1] == list(range(100))
    with bridge(server, group_id="other", auto_offset_reset="latest") as br:
        assert {s["start_offset"] for s in br.stats()} == {100}


def test_control_batches_are_dropped_and_skipped(broker, server):
    """Transaction markers occupy offsets but carry no data: the replica drops them, consumers
    read across the gap they leave."""
    broker.create_topic("t", 1)
    pidx = broker.pidx("t", 0)
    broker.produce("t", [b"a", b"b"], partition=0)                     # offsets 0, 1
    broker.native.ingest_bytes(pidx, control_batch(2), keep_control=True)  # offset 2
    broker.produce("t", [b"c"], partition=0)                           # offset 3
    broker.native.ingest_bytes(pidx, control_batch(4), keep_control=True)  # offset 4 (trailing)
    assert broker.end_offset("t", 0) == 5
    # the source broker's own consumers skip markers too
    c = KafkaConsumer("t", bootstrap_servers=broker.url, auto_offset_reset="earliest", consumer_timeout_ms=200)
    assert [(r.offset, r.value) for r in c] == [(0, b"a"), (1, b"b"), (3, b"c")]
    c.close()
    with bridge(server, group_id="g") as br:
        assert br.wait_caught_up(10)
        st = br.stats()[0]
        assert st["control_batches"] == 2 and st["batches"] == 2 and st["fetch_offset"] == 5
        c = KafkaConsumer("t", bootstrap_servers=br.url, group_id="g", auto_offset_reset="earliest",
                          enable_auto_commit=False, consumer_timeout_ms=200)
        assert [(r.offset, r.value) for r in c] == [(0, b"a"), (1, b"b"), (3, b"c")]
        c.commit()
        c.close()
        br.flush()
    assert broker.committed("g", "t", 0) == 4


def test_not_leader_and_commit_errors_recover(broker, server):
    broker.create_topic("t", 2)
    broker.fill("t", 100, "fixed_f32", size=8, records_per_batch=10)
    server.inject_fetch_errors("t", 1, NOT_LEADER, n=3)
    server.inject_commit_errors(n=2)
    with bridge(server, group_id="g", commit_interval_ms=2) as br:
        assert br.wait_caught_up(10)
        assert br.errors >= 3
        br.local.commit("g", {TopicPartition("t", 0): 60, TopicPartition("t", 1): 70})
        assert wait_for(lambda: broker.committed_offsets("g", "t") == {0: 60, 1: 70})


def test_flow_control_bounds_uncommitted_bytes(broker, server):
    broker.create_topic("t", 1)
    broker.fill("t", 2000, "fixed_f32", size=64, records_per_batch=20)  # ~550 KB
    with bridge(server, group_id="g", max_lag_bytes=64 << 10, max_partition_fetch_bytes=16 << 10,
                fetch_max_bytes=16 << 10) as br:
        assert wait_for(lambda: br.stats()[0]["throttled"] > 0)
        held = br.local.native.log_bytes(br.local.pidx("t", 0))
        assert held < (64 << 10) + (16 << 10) + 8192
        assert br.stats()[0]["fetch_offset"] < 2000
        br.local.commit("g", {TopicPartition("t", 0): br.stats()[0]["fetch_offset"]})
        assert wait_for(lambda: br.local.native.log_bytes(br.local.pidx("t", 0)) > held)


class Vec8(KafkaDataset):
    schema = FixedWidth(torch.float32, (8,))


@pytest.mark.parametrize("workers", [0, 2])
def test_device_loader_over_the_bridge_commits_to_the_cluster(broker, server, workers):
    """The flagship path end to end on CPU: cluster -> replica -> DeviceLoader -> auto_commit ->
    OffsetCommit.  Every record once, values intact, the cluster's committed offsets at the end."""
    broker.create_topic("t", 3)
    broker.fill("t", 90, "fixed_f32", size=8, records_per_batch=15)
    with bridge(server, group_id="trainer") as br:
        ckw = dict(bootstrap_servers=br.url, group_id="trainer", auto_offset_reset="earliest",
                   consumer_timeout_ms=400)
        if workers == 0:  # single-process mode: the dataset owns its consumer
            dl = DeviceLoader(Vec8("t", **ckw), 12, device="cpu", num_workers=0)
        else:
            dl = DeviceLoader(Vec8.placeholder(), 12, device="cpu", num_workers=workers,
                              worker_init_fn=Vec8.init_worker("t", **ckw))
        seen = set()
        for x in auto_commit(dl):
            for row in x.tolist():
                o, p = int(row[0]), int(row[1])
                assert row[2:] == [synth_f32(p, o, j) for j in range(2, 8)]
                seen.add((p, o))
        assert seen == {(p, o) for p in range(3) for o in range(90)}
    # close() flushed the final commit to the cluster
    assert broker.committed_offsets("trainer", "t") == {0: 90, 1: 90, 2: 90}


def test_bridge_partition_subset_per_rank(broker, server):
    broker.create_topic("t", 4)
    broker.fill("t", 20, "fixed_f32", size=8, records_per_batch=5)
    with bridge(server, partitions=[1, 3]) as br:
        assert br.wait_caught_up(10)
        assert [s["partition"] for s in br.stats()] == [1, 3]
        assert br.local.end_offset("t", 1) == 20 and br.local.end_offset("t", 0) == 0


def test_unreachable_cluster_raises():
    with pytest.raises(Exception, match="NoBrokersAvailable"):
        KafkaBridge("127.0.0.1:1", "t", url=f"shm://tkbr-none-{os.getpid()}", request_timeout_ms=500)


def test_committed_log_bytes_are_released(broker, server):
    """A replica frees what its group committed: log start moves up, the bytes below are punched
    out of the shm file (st_blocks drops), consumers carry on from the committed offset."""
    broker.create_topic("t", 1)
    broker.fill("t", 10000, "fixed_f32", size=256, records_per_batch=64)  # ~10.3 MB
    with bridge(server, group_id="g", release_bytes=2 << 20, log_capacity=64 << 20) as br:
        assert br.wait_caught_up(10)
        pidx = br.local.pidx("t", 0)
        path = os.path.join(br.local.dir, f"p{pidx:05d}.log")
        before = os.stat(path).st_blocks * 512
        assert before >= 9 << 20
        dl = DeviceLoader(Vec256.placeholder(), 256, device="cpu", num_workers=1,
                          worker_init_fn=Vec256.init_worker("t", bootstrap_servers=br.url, group_id="g",
                                                            auto_offset_reset="earliest", consumer_timeout_ms=300))
        n = sum(x.shape[0] for x in auto_commit(dl))
        assert n == 10000
        assert wait_for(lambda: br.stats()[0]["released"] >= 6 << 20)
        assert os.stat(path).st_blocks * 512 <= before - (6 << 20)
        assert br.local.beginning_offset("t", 0) > 0
    assert broker.committed("g", "t", 0) == 10000


class Vec256(KafkaDataset):
    schema = FixedWidth(torch.float32, (256,))
