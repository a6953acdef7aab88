"""ConsumerRebalanceListener (kafka-python's rebalance callbacks) on both consumer routes.

The reference hands every kwarg to kafka-python and lets users override ``new_consumer``
(/root/reference/README.md:46-57, src/kafka_dataset.py:188-206), so a user can subscribe with a
listener; kafka-python 2.0.2 calls ``on_partitions_revoked`` (whole assignment, eager protocol)
before every join and ``on_partitions_assigned`` after it.  Checked here:
  * the synthetic broker's group coordinator: a second member joining makes the first one see
    revoke(old) then assign(new), in that order, with the offsets it committed visible at revoke;
  * a DataLoader worker whose records the user finished: those are committed BEFORE the listener
    hears of the revocation (the commit channel is a revoke hook);
  * the Kafka-protocol route (KafkaBridge group membership): revoke/assign follow the bridges'
    assignment epochs;
  * listener type checking and a listener that raises (logged, iteration continues).
"""
import threading
import time

import pytest

from torchkafka_amd import ConsumerRebalanceListener, KafkaConsumer


class Recorder(ConsumerRebalanceListener):
    def __init__(self, consumer_ref=None, group=None, broker=None):
        self.events = []
        self.consumer_ref = consumer_ref
        self.group, self.broker = group, broker

    def on_partitions_revoked(self, revoked):
        committed = None
        if self.broker is not None:
            committed = {p: o for p, o in self.broker.committed_offsets(self.group, "t").items() if o is not None}
        self.events.append(("revoked", sorted(tp.partition for tp in revoked), committed))

    def on_partitions_assigned(self, assigned):
        self.events.append(("assigned", sorted(tp.partition for tp in assigned), None))


def _poll_until(c, cond, timeout=20.0):
    t0 = time.monotonic()
    while not cond() and time.monotonic() - t0 < timeout:
        c.poll(timeout_ms=20)
    return cond()


def test_listener_sees_revoke_then_assign_when_a_member_joins(broker):
    broker.create_topic("t", 4)
    broker.fill("t", 100, "fixed_f32", size=4, records_per_batch=10)
    kw = dict(bootstrap_servers=broker.url, group_id="g", auto_offset_reset="earliest", enable_auto_commit=False)
    a = KafkaConsumer(**kw)
    la = Recorder(group="g", broker=broker)
    a.subscribe(["t"], listener=la)
    assert _poll_until(a, lambda: len(a.assignment()) == 4)
    assert [e[:2] for e in la.events] == [("revoked", []), ("assigned", [0, 1, 2, 3])]
    got = a.poll(timeout_ms=200, max_records=50)
    assert got
    a.commit()
    committed_before = {p: o for p, o in broker.committed_offsets("g", "t").items() if o is not None}
    assert committed_before
    # a second member joins: both must poll for the rebalance to complete
    b = KafkaConsumer(**kw)
    lb = Recorder()
    b.subscribe(["t"], listener=lb)
    stop = threading.Event()

    def poll_b():
        while not stop.is_set():
            b.poll(timeout_ms=20)
    th = threading.Thread(target=poll_b)
    th.start()
    try:
        assert _poll_until(a, lambda: len(a.assignment()) == 2 and len(b.assignment()) == 2)
    finally:
        stop.set()
        th.join()
    kinds = [e[0] for e in la.events]
    assert kinds == ["revoked", "assigned", "revoked", "assigned"], la.events
    assert la.events[2][1] == [0, 1, 2, 3]                # the whole old assignment (eager)
    assert la.events[2][2] == committed_before            # what a committed is visible at revoke time
    assert len(la.events[3][1]) == 2
    assert set(la.events[3][1]) | set(lb.events[-1][1]) == {0, 1, 2, 3}
    assert [e[0] for e in lb.events] == ["revoked", "assigned"] and lb.events[0][1] == []
    a.close()
    b.close()


def test_listener_type_is_checked_and_a_failing_listener_is_logged(broker, caplog):
    broker.create_topic("t", 2)
    broker.fill("t", 10, "fixed_f32", size=4)
    c = KafkaConsumer(bootstrap_servers=broker.url, group_id="g2", auto_offset_reset="earliest")
    with pytest.raises(TypeError, match="ConsumerRebalanceListener"):
        c.subscribe(["t"], listener=object())

    class Bad(ConsumerRebalanceListener):
        def on_partitions_revoked(self, revoked):
            raise RuntimeError("boom")

        def on_partitions_assigned(self, assigned):
            raise RuntimeError("boom")

    c.subscribe(["t"], listener=Bad())
    with caplog.at_level("ERROR"):
        recs = []
        t0 = time.monotonic()
        while len(recs) < 20 and time.monotonic() - t0 < 20:
            for rs in c.poll(timeout_ms=50).values():
                recs += rs
    assert len(recs) == 20  # iteration carried on
    msgs = [r.getMessage() for r in caplog.records]
    assert any("failed on partition revocation" in m for m in msgs)
    assert any("failed on partition assignment" in m for m in msgs)
    c.close()


class _ListenedDataset:
    pass


def test_worker_commits_finished_batches_before_the_listener_hears_of_revocation(broker, tmp_path):
    """A DataLoader worker (reference multi-worker mode) subscribed with a listener: when another
    member joins, the batches the user finished are committed first (the commit channel is a revoke
    hook), so the listener's view of the committed offsets at revoke time covers them."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    broker.create_topic("t", 2)
    broker.fill("t", 400, "fixed_f32", size=4, records_per_batch=10)
    out = tmp_path / "events.json"
    env = dict(os.environ, PYTHONPATH=root)
    env.pop("WORLD_SIZE", None)
    p = subprocess.Popen([sys.executable, os.path.join(root, "tests", "helpers", "listener_member.py"), broker.url,
                          str(out)], cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        t0 = time.monotonic()
        while not (tmp_path / "events.json.ready").exists() and time.monotonic() - t0 < 60:
            time.sleep(0.05)
        assert (tmp_path / "events.json.ready").exists(), p.stderr.read() if p.poll() is not None else "not ready"
        joiner = KafkaConsumer(bootstrap_servers=broker.url, group_id="gl", auto_offset_reset="latest",
                               enable_auto_commit=False)
        joiner.subscribe(["t"])
        t0 = time.monotonic()
        while not joiner.assignment() and time.monotonic() - t0 < 30:
            joiner.poll(timeout_ms=20)
        assert joiner.assignment()
        joiner.close()  # leaves: another rebalance, the worker gets both partitions back
        stdout, stderr = p.communicate(timeout=120)
        assert p.returncode == 0, stderr[-3000:]
    finally:
        if p.poll() is None:
            p.kill()
    ev = json.load(open(out))
    kinds = [e["kind"] for e in ev["events"]]
    assert kinds[:2] == ["revoked", "assigned"] and kinds.count("revoked") >= 2, ev
    second = [e for e in ev["events"] if e["kind"] == "revoked"][1]
    # every record of every batch the user had finished when the rebalance began is committed
    fin = second["finished"]
    for p_, off in fin.items():
        assert (second["committed"].get(p_) or 0) >= off, second
