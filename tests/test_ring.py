"""The shared-memory slot ring: FIFO per worker, futex hand-offs, shutdown, worker-side packing."""
import multiprocessing as mp
import os
import time
import uuid

import pytest
import torch

from torchkafka_amd.ops.native import core


@pytest.fixture
def ring():
    r = core().Ring.create(f"/tktest-ring-{os.getpid()}-{uuid.uuid4().hex[:8]}", 2, 3, 4096)
    try:
        yield r
    finally:
        r.shutdown()
        r.unlink()


def _producer(ring_name, w, n):
    r = core().Ring.open(ring_name)
    for i in range(n):
        assert r.worker_acquire(w, i % r.slots_per_worker, 5000)
        g = r.gslot(w, i % r.slots_per_worker)
        view = r.payload_view(g)
        t = torch.frombuffer(view, dtype=torch.int64, count=2)
        t[0], t[1] = w, i
        r.set_slot(g, 1, 0, 0, 16, 0, 0, 0, 1, [(w, i, i + 1, 1)])
        r.worker_publish(g)


def test_fifo_per_worker_and_release_wakeup(ring):
    ctx = mp.get_context("fork")
    ps = [ctx.Process(target=_producer, args=(ring.name, w, 20)) for w in range(2)]
    for p in ps:
        p.start()
    seen = {0: [], 1: []}
    while sum(map(len, seen.values())) < 40:
        g = ring.main_acquire(5000, False)
        assert g >= 0
        t = torch.frombuffer(ring.payload_view(g), dtype=torch.int64, count=2)
        w, i = int(t[0]), int(t[1])
        assert ring.watermarks(g) == [(w, i, i + 1, 1)]
        seen[w].append(i)
        ring.main_release(g)  # wakes the producer blocked on this slot
    for p in ps:
        p.join(10)
        assert p.exitcode == 0
    assert seen == {0: list(range(20)), 1: list(range(20))}


def test_in_order_round_robin(ring):
    for w in (1, 0):
        for i in range(2):
            assert ring.worker_acquire(w, i, 0)
            g = ring.gslot(w, i)
            ring.set_slot(g, 1, 0, 0, 0, 0, 0, 0, 0, [])
            ring.worker_publish(g)
    got = [ring.main_acquire(100, True) for _ in range(4)]
    assert got == [ring.gslot(0, 0), ring.gslot(1, 0), ring.gslot(0, 1), ring.gslot(1, 1)]


def test_timeout_and_all_done(ring):
    t0 = time.monotonic()
    assert ring.main_acquire(50, False) == -1
    assert time.monotonic() - t0 >= 0.04
    ring.mark_done(0)
    ring.mark_done(1)
    assert ring.main_acquire(50, False) == -2


def test_worker_acquire_blocks_until_release_and_shutdown(ring):
    for i in range(3):
        assert ring.worker_acquire(0, i, 0)
    # the slot is FILLING: a second acquire times out
    assert not ring.worker_acquire(0, 0, 30)
    ring.shutdown()
    assert not ring.worker_acquire(0, 0, -1)  # shutdown unblocks immediately
    assert ring.is_shutdown()


def test_error_slot_roundtrip(ring):
    assert ring.worker_acquire(1, 0, 0)
    g = ring.gslot(1, 0)
    ring.set_slot(g, 0, 0, 0, 0, 0, 0, 0, 0, [])
    ring.set_error(g, "boom")
    ring.worker_publish(g)
    g2 = ring.main_acquire(100, False)
    info = ring.slot_info(g2)
    assert info["error"] == "boom" and info["flags"] & core().SLOT_ERROR


def test_fill_slot_native_pack(broker):
    from torchkafka_amd.client import KafkaConsumer

    broker.create_topic("t", 2)
    broker.fill("t", 100, "fixed_f32", size=16, records_per_batch=30)
    r = core().Ring.create(f"/tktest-fill-{uuid.uuid4().hex[:8]}", 1, 2, 64 * 1024)
    try:
        c = KafkaConsumer(bootstrap_servers=broker.url, auto_offset_reset="earliest")
        c.assign_shard(["t"], 0, 1)
        f = c._fetcher
        assert r.worker_acquire(0, 0, 0)
        rows, scanned, timed_out, shut = f.fill_slot(r, 0, core().PACK_FIXED, 4, 16, 0, -1, True, False, 150, 50)
        assert rows == 150 and scanned == 150 and not timed_out and not shut
        x = torch.frombuffer(r.payload_view(0), dtype=torch.float32, count=150 * 16).view(150, 16)
        assert sorted(map(tuple, x[:, :2].long().tolist())) == sorted(
            [(o, 0) for o in range(100)] + [(o, 1) for o in range(50)]) or \
            sorted(map(tuple, x[:, :2].long().tolist())) == sorted(
            [(o, 1) for o in range(100)] + [(o, 0) for o in range(50)])
        wm = {p: (first, nxt, cnt) for p, first, nxt, cnt in r.watermarks(0)}
        assert sum(v[2] for v in wm.values()) == 150
        # the rest: 50 rows, then the stream idles -> timed out
        assert r.worker_acquire(0, 1, 0)
        rows, _, timed_out, _ = f.fill_slot(r, 1, core().PACK_FIXED, 4, 16, 0, -1, True, False, 150, 50)
        assert rows == 50 and timed_out
    finally:
        r.unlink()


def test_gather_slot_locates_every_value_in_the_log(broker):
    """kPackGatherFixed (h2d='direct'): one (pidx << 44 | byte offset) per row, pointing at exactly
    the record value the copying packer would have written, with per-partition log extents."""
    import struct

    from torchkafka_amd.client.consumer import KafkaConsumer
    from torchkafka_amd.ops.native import core

    broker.create_topic("g", 3)
    rng = __import__("random").Random(5)
    for p in range(3):
        vals = [bytes(rng.getrandbits(8) for _ in range(40)) for _ in range(30)]
        keys = [b"k" * rng.randrange(0, 7) for _ in range(30)]  # vary the value alignment in the log
        broker.produce("g", vals, partition=p, keys=keys)
    ring = core().Ring.create(f"/tkgather-{os.getpid()}", 1, 2, 1 << 16)
    try:
        c = KafkaConsumer("g", bootstrap_servers=broker.url, group_id="x", auto_offset_reset="earliest")
        c.assign_shard(["g"], 0, 1, 0, 1)
        assert ring.worker_acquire(0, 0, 1000)
        g = ring.gslot(0, 0)
        rows, scanned, _, _ = c._fetcher.fill_slot(ring, g, core().PACK_FIXED, 4, 10, 0, -1, True, False, 64, 100,
                                                    True)
        assert rows == 64
        summ = ring.slot_summary(g)
        assert summ[7] == core().PACK_GATHER_FIXED and summ[2] == 64 * 8
        ents = struct.unpack("<64Q", bytes(ring.payload_view(g)[: 64 * 8]))
        b = broker.native
        tps = {broker.pidx("g", p): p for p in range(3)}
        got = [(tps[e >> 44], e & ((1 << 44) - 1)) for e in ents]
        # reference: the same records through the copying consumer path
        c2 = KafkaConsumer("g", bootstrap_servers=broker.url, group_id="y", auto_offset_reset="earliest",
                           consumer_timeout_ms=100)
        c2.assign_shard(["g"], 0, 1, 0, 1)
        by_tp = {}
        for r in c2:
            by_tp.setdefault(r.partition, []).append(r.value)
        seen = {p: 0 for p in range(3)}
        for p, off in got:
            assert b.read_log(broker.pidx("g", p), off, 40) == by_tp[p][seen[p]]
            seen[p] += 1
        ext = dict(zip([w[0] for w in ring.watermarks(g)], ring.slot_info(g).get("log_end", [])))
        for pidx, end in ext.items():
            assert end == max(off + 40 for p, off in got if broker.pidx("g", p) == pidx)
    finally:
        ring.shutdown()
        ring.unlink()
