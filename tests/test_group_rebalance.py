"""Group-managed partition assignment on the reference API path (CPU, Kafka-protocol test cluster).

In the reference every DataLoader worker's ``KafkaConsumer(*topics, group_id=...)`` is a member of
the consumer group, so the group coordinator splits the partitions among all consumers of all
processes and rebalances them as members come and go (/root/reference/src/kafka_dataset.py:206,
219-231).  Here the same API over a cluster reached through the native client: each
consumer's KafkaBridge joins the group and follows rebalances in process.

Checked against this repo's own Kafka-protocol server (parity with a real broker is unpinned):
  * two independent processes in one group consume disjoint partitions, every record exactly once;
  * a third process joining mid-stream triggers a rebalance: every record is delivered at least
    once, and no partition's committed offset at the cluster ever moves backwards.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from torchkafka_amd.broker import KafkaWireServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MEMBER = os.path.join(ROOT, "tests", "helpers", "group_member.py")


def _spawn(addr, nw=0, slow=0.0, idle=4000, mode="ref"):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    return subprocess.Popen([sys.executable, MEMBER, addr, str(nw), str(slow), str(idle), mode], cwd=ROOT, env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def _result(proc, timeout=120):
    out, err = proc.communicate(timeout=timeout)
    assert proc.returncode == 0, err[-4000:]
    lines = [json.loads(x) for x in out.splitlines() if x.startswith('{"seen"')]
    assert len(lines) == 1, (out[-2000:], err[-2000:])
    return [tuple(x) for x in lines[0]["seen"]]


def _monotone(commit_log):
    last = {}
    for group, topic, p, off in commit_log:
        key = (group, topic, p)
        assert off >= last.get(key, -1), f"committed offset of {key} moved back: {last[key]} -> {off}"
        last[key] = off
    return last


@pytest.fixture(params=["legacy", "kafka4"])
def cluster(broker, request):
    srv = KafkaWireServer(broker, profile=request.param).start()
    try:
        yield srv
    finally:
        srv.close()


def test_two_processes_in_one_group_split_the_partitions(broker, cluster):
    broker.create_topic("t", 6)
    broker.fill("t", 300, "fixed_f32", size=8, records_per_batch=20)
    cluster.join_delay_s = 6.0  # the first round waits for both processes (their imports take a while)
    procs = [_spawn(cluster.address), _spawn(cluster.address)]
    seen = [_result(p) for p in procs]
    parts = [{p for p, _ in s} for s in seen]
    assert parts[0] and parts[1] and not parts[0] & parts[1], parts  # disjoint shares
    assert parts[0] | parts[1] == set(range(6))
    allrec = seen[0] + seen[1]
    assert len(allrec) == len(set(allrec)) == 6 * 300  # every record exactly once
    assert broker.committed_offsets("g", "t") == {p: 300 for p in range(6)}
    _monotone(cluster.commit_log)
    assert cluster.group_members("g") == {}  # both left the group


def test_a_third_process_joining_rebalances_at_least_once(broker, cluster):
    import threading

    broker.create_topic("t", 6)
    broker.fill("t", 400, "fixed_f32", size=8, records_per_batch=10)
    cluster.join_delay_s = 6.0
    # a long idle: under a loaded host the joiner can take longer to start than the feed lasts
    a, b = _spawn(cluster.address, slow=0.01, idle=30000), _spawn(cluster.address, slow=0.01, idle=30000)
    t0 = time.monotonic()
    while len(cluster.commit_log) < 6 and time.monotonic() - t0 < 60:
        time.sleep(0.05)
    assert cluster.commit_log, "the first two members never committed"
    # a live stream while a third process (two DataLoader workers: two more group members) joins
    def produce():
        for _ in range(40):
            broker.fill("t", 5, "fixed_f32", size=8, records_per_batch=5)
            time.sleep(0.1)
    feed = threading.Thread(target=produce)
    feed.start()
    c = _spawn(cluster.address, nw=2, slow=0.01, idle=8000)
    t0 = time.monotonic()
    while len(cluster.group_members("g")) < 4 and time.monotonic() - t0 < 60:
        time.sleep(0.05)
    feed.join()
    assert len(cluster.group_members("g")) == 4, cluster.group_members("g")
    broker.fill("t", 100, "fixed_f32", size=8, records_per_batch=10)  # after the rebalance: every member gets some
    seen = [_result(p, timeout=240) for p in (a, b, c)]
    allrec = set(seen[0]) | set(seen[1]) | set(seen[2])
    assert allrec == {(p, o) for p in range(6) for o in range(700)}  # at least once
    assert {p for p, _ in seen[2]}, "the late member never got a partition"
    last = _monotone(cluster.commit_log)
    assert {p: last[("g", "t", p)] for p in range(6)} == {p: 700 for p in range(6)}
    dup = len(seen[0]) + len(seen[1]) + len(seen[2]) - len(allrec)
    assert dup < 6 * 700 // 4, dup  # re-deliveries only around the rebalances


def test_device_loader_workers_follow_a_rebalance(broker, cluster):
    """DeviceLoader workers (the native fetch loop) as group members: a process joining mid-stream
    takes partitions from them, and their fills pick up the new assignment."""
    import threading

    broker.create_topic("t", 4)
    broker.fill("t", 200, "fixed_f32", size=8, records_per_batch=10)
    cluster.join_delay_s = 5.0
    # a long idle: under a loaded host the joiner can take longer to start than the feed lasts
    a = _spawn(cluster.address, nw=2, slow=0.01, idle=30000, mode="device")
    t0 = time.monotonic()
    while len(cluster.commit_log) < 4 and time.monotonic() - t0 < 60:
        time.sleep(0.05)
    assert cluster.commit_log, "the DeviceLoader workers never committed"

    def produce():
        for _ in range(30):
            broker.fill("t", 5, "fixed_f32", size=8, records_per_batch=5)
            time.sleep(0.1)
    feed = threading.Thread(target=produce)
    feed.start()
    b = _spawn(cluster.address, slow=0.01, idle=8000)
    t0 = time.monotonic()
    while len(cluster.group_members("g")) < 3 and time.monotonic() - t0 < 60:
        time.sleep(0.05)
    feed.join()
    assert len(cluster.group_members("g")) == 3
    broker.fill("t", 50, "fixed_f32", size=8, records_per_batch=10)
    seen = [_result(p, timeout=240) for p in (a, b)]
    allrec = set(seen[0]) | set(seen[1])
    assert allrec == {(p, o) for p in range(4) for o in range(400)}  # at least once
    assert {p for p, _ in seen[1]}, "the joining member never got a partition"
    last = _monotone(cluster.commit_log)
    assert {p: last[("g", "t", p)] for p in range(4)} == {p: 400 for p in range(4)}
