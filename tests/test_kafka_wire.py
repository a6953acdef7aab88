"""Kafka wire protocol: the native replicator (KafkaBridge) against a Kafka-protocol server (CPU).

The reference consumes a real cluster through kafka-python (/root/reference/src/kafka_dataset.py:
21-22, 206).  No cluster exists here, so `KafkaWireServer` serves a synthetic broker over the
Kafka protocol (ApiVersions, Metadata, ListOffsets, Fetch, FindCoordinator, OffsetCommit,
OffsetFetch, the group APIs, SASL) at a "legacy" (pre-2.x) and a "kafka4" (KIP-896) version
profile, and the native replicator (csrc/core/replicator.cpp) mirrors it into a local
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
from torchkafka_amd.broker.wire_server import NOT_LEADER, PROFILES as KW_PROFILES, control_batch
from torchkafka_amd.client.records import TopicPartition
from torchkafka_amd.ops.native import core


@pytest.fixture(params=["legacy", "kafka4"])
def server(broker, request):
    """The test cluster at both protocol profiles: a pre-2.x broker (the versions the client used
    to hard-code) and Kafka 4.x after KIP-896 (the pre-2.1 request versions removed)."""
    srv = KafkaWireServer(broker, profile=request.param).start()
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
                fetch_max_bytes=16 << 10, ring_bytes=0) as br:  # a linear log: max_lag_bytes bounds it
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
    with bridge(server, group_id="g", release_bytes=2 << 20, release_step=2 << 20, log_capacity=64 << 20,
                ring_bytes=0) as br:
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
        assert wait_for(lambda: br.stats()[0]["released"] >= 6 << 20), br.stats()
        assert os.stat(path).st_blocks * 512 <= before - (6 << 20)
        assert br.local.beginning_offset("t", 0) > 0
    assert broker.committed("g", "t", 0) == 10000


class Vec256(KafkaDataset):
    schema = FixedWidth(torch.float32, (256,))


# ---------------------------------------------------------------- compressed record sets
# Minimal encoders (the image has no snappy/lz4 packages): greedy 4-byte matches, enough to
# exercise every element type of the native decoders (literals of every length class, copies
# with overlapping matches).

def _snappy_raw(data: bytes) -> bytes:
    out = bytearray()
    n = len(data)
    v = n
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    table, i, lit = {}, 0, 0

    def emit_literal(a, b):
        while a < b:
            k = min(b - a, 65536)
            if k <= 60:
                out.append((k - 1) << 2)
            elif k <= 256:
                out.extend(bytes([60 << 2, k - 1]))
            else:
                out.extend(bytes([61 << 2]) + (k - 1).to_bytes(2, "little"))
            out.extend(data[a:a + k])
            a += k

    while i + 4 <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None and i - j < 65536:
            m = 4
            while i + m < n and data[j + m] == data[i + m] and m < 64:
                m += 1
            emit_literal(lit, i)
            off = i - j
            if m <= 11 and off < 2048:
                out += bytes([1 | ((m - 4) << 2) | ((off >> 8) << 5), off & 0xFF])
            else:
                out += bytes([2 | ((m - 1) << 2)]) + off.to_bytes(2, "little")
            i += m
            lit = i
        else:
            i += 1
    emit_literal(lit, n)
    return bytes(out)


def _xerial(data: bytes, block=32 << 10) -> bytes:
    out = bytearray(b"\x82SNAPPY\x00" + (1).to_bytes(4, "big") + (1).to_bytes(4, "big"))
    for a in range(0, len(data), block):
        c = _snappy_raw(data[a:a + block])
        out += len(c).to_bytes(4, "big") + c
    return bytes(out)


def _lz4_block(data: bytes) -> bytes:
    out = bytearray()
    n, i, lit, table = len(data), 0, 0, {}

    def lenbytes(v):
        b = bytearray()
        while v >= 255:
            b.append(255)
            v -= 255
        b.append(v)
        return b

    while i + 12 <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None and i - j < 65536:
            m = 4
            while i + m < n - 5 and data[j + m] == data[i + m]:
                m += 1
            ll, ml = i - lit, m - 4
            out.append((min(ll, 15) << 4) | min(ml, 15))
            if ll >= 15:
                out += lenbytes(ll - 15)
            out += data[lit:i]
            out += (i - j).to_bytes(2, "little")
            if ml >= 15:
                out += lenbytes(ml - 15)
            i += m
            lit = i
        else:
            i += 1
    ll = n - lit
    out.append(min(ll, 15) << 4)
    if ll >= 15:
        out += lenbytes(ll - 15)
    out += data[lit:]
    return bytes(out)


def _lz4_frame(data: bytes, block=64 << 10) -> bytes:
    out = bytearray((0x184D2204).to_bytes(4, "little") + bytes([0x60, 0x40, 0x82]))  # FLG, BD, HC
    for a in range(0, len(data), block):
        chunk = data[a:a + block]
        c = _lz4_block(chunk)
        if len(c) >= len(chunk):
            out += (len(chunk) | 0x80000000).to_bytes(4, "little") + chunk
        else:
            out += len(c).to_bytes(4, "little") + c
    out += (0).to_bytes(4, "little")
    return bytes(out)


def _zstd(data: bytes) -> bytes:
    """zstd frames from the system libzstd (ctypes): two concatenated frames, as a streaming
    producer that flushes mid-batch leaves them."""
    import ctypes
    try:
        z = ctypes.CDLL("libzstd.so.1")
    except OSError:
        pytest.skip("libzstd.so.1 not loadable")
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    out = b""
    for part in (data[:len(data) // 3], data[len(data) // 3:]):
        cap = z.ZSTD_compressBound(ctypes.c_size_t(len(part)))
        buf = ctypes.create_string_buffer(cap)
        n = z.ZSTD_compress(buf, cap, part, len(part), 3)
        assert n < cap
        out += buf.raw[:n]
    return out


CODECS = {1: None, 2: _xerial, 3: _lz4_frame, 4: _zstd}


def _codec(codec):
    import gzip
    return gzip.compress if codec == 1 else CODECS[codec]


def _compress_batch(batch: bytes, codec: int) -> bytes:
    import struct

    records = batch[61:]
    comp = _codec(codec)(records)
    hdr = bytearray(batch[:61])
    attrs = struct.unpack_from(">h", hdr, 21)[0] | codec
    struct.pack_into(">h", hdr, 21, attrs)
    struct.pack_into(">i", hdr, 8, 61 - 12 + len(comp))
    body = bytes(hdr[21:]) + comp
    struct.pack_into(">I", hdr, 17, core().crc32c(body))
    return bytes(hdr[:21]) + body


@pytest.mark.parametrize("codec", [1, 2, 3, 4])
def test_native_decompressors(codec):
    data = (b"abcabcabcabc" * 300 + bytes(range(256)) * 40 + b"x" * 5000 + os.urandom(3000)) * 3
    comp = _codec(codec)(data)
    assert core().decompress(codec, comp) == data
    assert core().decompress(2, _snappy_raw(data)) == data  # raw snappy (no xerial framing)
    with pytest.raises(Exception, match="corrupt compressed|CRC|Corrupt"):
        core().decompress(codec, comp[: len(comp) // 2])


def test_zstd_goes_through_the_system_library():
    assert core().zstd_available()  # libzstd.so.1 ships with the image
    with pytest.raises(Exception, match="corrupt compressed"):
        core().decompress(4, b"\x28\xb5\x2f\xfd")  # bare magic: a truncated frame
    with pytest.raises(Exception, match="UnsupportedCodecError"):
        core().decompress(5, b"xyz")


@pytest.mark.parametrize("codec", [1, 2, 3, 4])
def test_compressed_batches_are_inflated_on_ingest(broker, server, codec):
    """A producer's compressed batches reach the replica as plain RecordBatch v2 (fresh CRC), so
    the loader and the device decoders read them like any other batch."""
    ref = SyntheticBroker.create(f"shm://tkref-{os.getpid()}-{uuid.uuid4().hex[:6]}", log_capacity=64 << 20)
    try:
        ref.create_topic("t", 1)
        ref.fill("t", 600, "fixed_f32", size=64, records_per_batch=40)
        raw = log_bytes(ref, "t", 0)
        broker.create_topic("t", 1)
        pidx = broker.pidx("t", 0)
        o = 0
        while o < len(raw):
            blen = int.from_bytes(raw[o + 8:o + 12], "big") + 12
            broker.native.ingest_bytes(pidx, _compress_batch(raw[o:o + blen], codec), keep_control=True)
            o += blen
        assert broker.end_offset("t", 0) == 600
        assert len(log_bytes(broker, "t", 0)) < len(raw)  # stored compressed at the source
        with bridge(server, group_id="g") as br:
            assert br.wait_caught_up(10)
            assert log_bytes(br.local, "t", 0) == raw       # inflated replica == uncompressed log
            dl = DeviceLoader(Vec64.placeholder(), 50, device="cpu", num_workers=1,
                              worker_init_fn=Vec64.init_worker("t", bootstrap_servers=br.url, group_id="g",
                                                               auto_offset_reset="earliest",
                                                               consumer_timeout_ms=300))
            rows = torch.cat(list(auto_commit(dl)))
            assert rows.shape == (600, 64)
            assert rows[:, 0].tolist() == [float(i) for i in range(600)]
            assert rows[7, 2:].tolist() == [synth_f32(0, 7, j) for j in range(2, 64)]
    finally:
        ref.destroy()


@pytest.mark.parametrize("compression", ["lz4", "zstd", "gzip"])
def test_compressed_topic_streams_through_a_ring_replica(broker, server, compression):
    """A compressed topic larger than the replica's ring, fetched in small record sets: after the
    first set shows the partition is compressed, each fetch thread hands its sets to an inflater
    and asks for the next while it inflates (replicator.cpp inflate_one), and the ring waits for
    the consumer's commits.  Every record arrives once, in order, per partition."""
    broker.create_topic("src", 2)
    broker.fill("src", 3000, "fixed_f32", size=64, records_per_batch=40)  # ~840 KiB per partition
    broker.create_topic("t", 2)
    info = broker.copy_compressed("src", "t", compression)
    assert info["compressed_bytes"] < info["raw_bytes"] and info["batches"] == 2 * 75
    with bridge(server, group_id="g", ring_bytes=256 << 10, max_partition_fetch_bytes=32 << 10) as br:
        dl = DeviceLoader(Vec64.placeholder(), 50, device="cpu", num_workers=2,
                          worker_init_fn=Vec64.init_worker("t", bootstrap_servers=br.url, group_id="g",
                                                           auto_offset_reset="earliest", consumer_timeout_ms=1000))
        rows = torch.cat(list(auto_commit(dl)))
        st = br.stats()
        assert br.errors == 0, br.last_error()
    assert rows.shape == (6000, 64)
    for part in (0, 1):
        offs = rows[rows[:, 1] == part][:, 0].tolist()
        assert offs == [float(i) for i in range(3000)]
    assert sum(s["inflated_batches"] for s in st) == 150
    assert br._r.inflate_threads >= 1  # the pipelined path ran


def _batch_spans(raw: bytes) -> list[tuple[int, int]]:
    """(base offset, next offset) of every RecordBatch of a log, in log order."""
    out, o = [], 0
    while len(raw) - o >= 61:
        total = int.from_bytes(raw[o + 8:o + 12], "big") + 12
        base = int.from_bytes(raw[o:o + 8], "big")
        out.append((base, base + int.from_bytes(raw[o + 23:o + 27], "big") + 1))
        o += total
    return out


def _assert_contiguous(b: SyntheticBroker, topic: str, p: int, start: int, end: int) -> None:
    spans = _batch_spans(log_bytes(b, topic, p))
    assert spans, f"{topic}-{p}: empty replica"
    assert spans[0][0] <= start < spans[0][1] or spans[0][0] == start, (p, spans[0], start)
    for (_, n0), (b1, _) in zip(spans, spans[1:]):
        assert b1 == n0, f"{topic}-{p}: gap or overlap in the replica log at {n0} -> {b1}"
    assert spans[-1][1] == end, (p, spans[-1], end)


def _mixed_compressibility_topic(broker, topic: str, n_parts: int, n: int, noisy: range, codec: str) -> None:
    """Records f32[64] = (offset, partition, payload) in batches of 40, the payload zeros (lz4 /
    zstd shrink it ~10x) except for offsets in ``noisy``, random bytes (they grow when compressed): the
    inflation ratio the replicator learns crosses 1 and back while record sets are in flight."""
    import numpy as np

    rng = np.random.default_rng(7)
    broker.create_topic("src-" + topic, n_parts)
    for p in range(n_parts):
        for b0 in range(0, n, 40):
            rows = np.zeros((min(40, n - b0), 64), np.float32)
            rows[:, 0] = np.arange(b0, b0 + len(rows))
            rows[:, 1] = p
            for i, o in enumerate(range(b0, b0 + len(rows))):
                if o in noisy:  # random bytes: lz4 / zstd output is larger than its input
                    rows[i, 2:] = rng.integers(0, 256, 62 * 4, dtype=np.uint8).view(np.float32)
            broker.produce("src-" + topic, [r.tobytes() for r in rows], partition=p)
    broker.create_topic(topic, n_parts)
    broker.copy_compressed("src-" + topic, topic, codec)


@pytest.mark.parametrize("compression", ["lz4", "zstd"])
def test_compression_ratio_crossing_one_keeps_the_replica_in_order(broker, server, compression, monkeypatch):
    """while compressed record sets wait for the inflater, later sets are asked for
    from past them; a set that inflates to less than its wire size used to take the synchronous path
    and be stored first, and the inflater then dropped the earlier sets as already held -- a silent
    gap.  Every set now queues behind the ones in flight, so each partition's replica stays
    contiguous and every record arrives once, in order."""
    noisy = [o for o in range(3000) if (o // 120) % 2]  # the ratio crosses 1 every 3 batches
    # a slow inflater keeps kMaxInflight sets queued: the case that lost records
    monkeypatch.setenv("TORCHKAFKA_TEST_INFLATE_DELAY_US", "1500")
    _mixed_compressibility_topic(broker, "t", 2, 3000, noisy, compression)
    with bridge(server, group_id="g", ring_bytes=256 << 10, max_partition_fetch_bytes=16 << 10) as br:
        dl = DeviceLoader(Vec64.placeholder(), 50, device="cpu", num_workers=2,
                          worker_init_fn=Vec64.init_worker("t", bootstrap_servers=br.url, group_id="g",
                                                           auto_offset_reset="earliest", consumer_timeout_ms=1000))
        rows = torch.cat(list(auto_commit(dl)))
        assert br.errors == 0, br.last_error()
        assert br.out_of_order == 0
    assert rows.shape == (6000, 64)
    for part in (0, 1):
        offs = rows[rows[:, 1] == part][:, 0].tolist()
        assert offs == [float(i) for i in range(3000)]


def test_rebalance_while_compressed_sets_are_in_flight(broker, server):
    """a partition restarted by a rebalance while record sets asked for at its old
    position still wait for the inflater.  Those sets are dropped (assignment epoch and pipeline
    generation); each member's replica of each partition it owns ends up contiguous from where its
    ownership started to the end of the topic."""
    _mixed_compressibility_topic(broker, "t", 4, 6000, range(2000, 3000), "lz4")
    kw = dict(group_id="g", subscribe=True, heartbeat_interval_ms=20, session_timeout_ms=3000,
              max_partition_fetch_bytes=8 << 10, ring_bytes=0)  # linear logs: nobody consumes here
    first = bridge(server, **kw)
    try:
        assert sorted(first.assignment) == [0, 1, 2, 3]
        first.local.commit("g", {TopicPartition("t", p): 100 for p in range(4)})
        second = bridge(server, **kw)  # joins while first is still fetching the compressed topic
        try:
            assert wait_for(lambda: len(first.assignment) == 2, 5)
            assert first.wait_caught_up(20) and second.wait_caught_up(20)
            assert first.errors == 0 and second.errors == 0, (first.last_error(), second.last_error())
            for br in (first, second):
                for s in br.stats():
                    if s["owned"]:
                        _assert_contiguous(br.local, "t", s["partition"], s["start_offset"], 6000)
        finally:
            second.close()
        assert wait_for(lambda: sorted(first.assignment) == [0, 1, 2, 3], 5) and first.wait_caught_up(20)
        for s in first.stats():
            _assert_contiguous(first.local, "t", s["partition"], s["start_offset"], 6000)
        assert first.errors == 0, first.last_error()
    finally:
        first.close()


def test_ring_replica_grows_its_reservation_for_a_first_batch_that_inflates_past_it(broker, server):
    """A ring replica reserves room for a Fetch by the inflation ratio learnt so far (none at the
    start): a first compressed batch that inflates to more than max_partition_fetch_bytes never fit
    the reservation, and the partition stalled with nothing stored.  The reservation now doubles
    until the batch fits."""
    _mixed_compressibility_topic(broker, "t", 1, 400, range(0), "lz4")  # 457 B batches -> 10.7 KiB
    with bridge(server, group_id="g", ring_bytes=1 << 20, max_partition_fetch_bytes=4096) as br:
        assert wait_for(lambda: br.local.end_offset("t", 0) == 400, 10), br.stats()[0]
        assert br.errors == 0, br.last_error()
        _assert_contiguous(br.local, "t", 0, 0, 400)


def test_compress_round_trips_through_the_native_decoders():
    data = bytes(range(256)) * 300 + b"tail" * 1000
    for codec in (1, 3, 4):
        assert core().decompress(codec, core().compress(codec, data)) == data
    with pytest.raises(Exception, match="UnsupportedCodecError"):
        core().compress(2, data)  # no snappy encoder


def test_corrupt_compressed_batch_stops_the_partition(broker, server):
    ref = SyntheticBroker.create(f"shm://tkref-{os.getpid()}-{uuid.uuid4().hex[:6]}", log_capacity=64 << 20)
    try:
        ref.create_topic("t", 1)
        ref.fill("t", 40, "fixed_f32", size=16, records_per_batch=20)
        raw = log_bytes(ref, "t", 0)
        blen = int.from_bytes(raw[8:12], "big") + 12
        good = _compress_batch(raw[:blen], 1)
        bad = bytearray(_compress_batch(raw[blen:], 1))
        bad[-3] ^= 0xFF  # flips a compressed byte: the producer CRC no longer matches
        broker.create_topic("t", 1)
        pidx = broker.pidx("t", 0)
        broker.native.ingest_bytes(pidx, good, keep_control=True)
        broker.native.ingest_bytes(pidx, bytes(bad), keep_control=True)
        with bridge(server) as br:
            assert wait_for(lambda: br.errors > 0)
            assert "CRC" in br.last_error()
            assert br.local.end_offset("t", 0) == 20  # the good batch only
    finally:
        ref.destroy()


class Vec64(KafkaDataset):
    schema = FixedWidth(torch.float32, (64,))


def test_multi_node_cluster_fetches_from_each_leader(broker):
    """Three nodes, partition p led by node p % 3: the replicator opens one fetch thread per
    leader; a node asked for a partition it does not lead answers NOT_LEADER."""
    import socket as _s

    broker.create_topic("t", 6)
    broker.fill("t", 300, "fixed_f32", size=16, records_per_batch=30)
    socks = [_s.socket() for _ in range(3)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    cluster = [(i, "127.0.0.1", ports[i]) for i in range(3)]
    nodes = [KafkaWireServer(broker, port=ports[i], node_id=i, cluster=cluster).start() for i in range(3)]
    try:
        c = core().WireClient(nodes[0].address)
        assert [p[1] for p in c.metadata("t")[1]] == [0, 1, 2, 0, 1, 2]
        assert sorted(b[0] for b in c.brokers()) == [0, 1, 2]
        with bridge(nodes[2], group_id="g") as br:  # bootstrap through any node
            assert br.wait_caught_up(10)
            for p in range(6):
                assert log_bytes(br.local, "t", p) == log_bytes(broker, "t", p)
            assert br.errors == 0
            br.local.commit("g", {TopicPartition("t", p): 100 + p for p in range(6)})
            br.flush()
        assert broker.committed_offsets("g", "t") == {p: 100 + p for p in range(6)}
        fetched = [n.requests.get(1, 0) for n in nodes]
        assert all(f > 0 for f in fetched), fetched
    finally:
        for n in nodes:
            n.close()


def test_device_loader_bridges_a_cluster_named_like_the_reference(broker, server):
    """`init_worker('t', bootstrap_servers='host:port', group_id=...)` -- the reference's usage --
    works unchanged: the loader mirrors this rank's partitions through a KafkaBridge (bridge='auto')
    and its commits land in the cluster."""
    broker.create_topic("t", 4)
    broker.fill("t", 60, "fixed_f32", size=8, records_per_batch=12)
    dl = DeviceLoader(Vec8.placeholder(), 16, device="cpu", num_workers=2,
                      worker_init_fn=Vec8.init_worker("t", bootstrap_servers=[server.address], group_id="ref",
                                                      auto_offset_reset="earliest", consumer_timeout_ms=400))
    assert len(dl._bridges) == 1 and dl._servers.startswith("shm://")
    seen = set()
    for x in auto_commit(dl):
        seen |= {(int(p), int(o)) for o, p in x[:, :2].tolist()}
    dl.close()
    assert seen == {(p, o) for p in range(4) for o in range(60)}
    assert broker.committed_offsets("ref", "t") == {p: 60 for p in range(4)}


def test_bridge_off_gives_each_worker_its_own_consumer(broker, server):
    """bridge=False: no loader-level replica; every worker builds its consumer as the reference does
    (kafka-python when installed, else the native wire route with its own replica of the worker's
    partitions), and the workers' consumers commit."""
    broker.create_topic("t", 4)
    broker.fill("t", 30, "fixed_f32", size=8, records_per_batch=10)
    dl = DeviceLoader(Vec8.placeholder(), 10, device="cpu", num_workers=2, bridge=False,
                      worker_init_fn=Vec8.init_worker("t", bootstrap_servers=server.address, group_id="pw",
                                                      auto_offset_reset="earliest", consumer_timeout_ms=400))
    assert dl._bridges == [] and dl._sink == "worker"
    n = sum(x.shape[0] for x in auto_commit(dl))
    dl.close()
    assert n == 120
    assert wait_for(lambda: broker.committed_offsets("pw", "t") == {p: 30 for p in range(4)}), \
        broker.committed_offsets("pw", "t")


class Doubled(KafkaDataset):
    def _process(self, record):  # the reference's README example shape: bytes -> tensor
        v = torch.frombuffer(bytearray(record.value), dtype=torch.float32)
        return None if int(v[0]) % 5 == 4 else v[:2] * 2


@pytest.mark.parametrize("workers", [0, 2])
def test_reference_api_reads_a_cluster_without_kafka_python(broker, server, workers):
    """The reference's own usage -- KafkaDataset + torch DataLoader + auto_commit, pointed at
    'host:port' -- works without kafka-python: the native wire route mirrors each worker's share of
    the partitions and the commits reach the cluster (None-skipped records committed too, B6)."""
    from torch.utils.data import DataLoader

    broker.create_topic("t", 4)
    broker.fill("t", 40, "fixed_f32", size=8, records_per_batch=8)
    kw = dict(bootstrap_servers=[server.address], group_id="refgrp", auto_offset_reset="earliest",
              consumer_timeout_ms=500)
    if workers == 0:
        dl = DataLoader(Doubled("t", **kw), batch_size=4)
    else:
        dl = DataLoader(Doubled.placeholder(), batch_size=4, num_workers=workers,
                        worker_init_fn=Doubled.init_worker("t", **kw))
    rows = torch.cat(list(auto_commit(dl)))
    assert rows.shape == (4 * 32, 2)
    got = sorted((int(o) // 2, int(p) // 2) for o, p in rows.tolist())
    assert got == sorted((o, p) for p in range(4) for o in range(40) if o % 5 != 4)
    if workers == 0:
        dl.dataset.close()  # the reference's close() does not commit (R4): what auto_commit committed stays
    last = {p: max(o for o, q in got if q == p) for p in range(4)}

    def covered():
        c = broker.committed_offsets("refgrp", "t")
        return all(c[p] is not None and c[p] >= last[p] + 1 for p in range(4))
    # every delivered record is committed in the cluster (a trailing None-skipped record may wait for
    # the next commit, B6)
    assert wait_for(covered), (broker.committed_offsets("refgrp", "t"), last)


def test_replicator_reconnects_after_the_broker_restarts(broker):
    """The cluster goes away mid-stream and comes back on the same address: the fetch threads
    back off, reconnect, refresh metadata and carry on from where the replica ends."""
    broker.create_topic("t", 2)
    broker.fill("t", 100, "fixed_f32", size=8, records_per_batch=10)
    srv = KafkaWireServer(broker).start()
    port = srv.port
    br = bridge(srv, group_id="g")
    try:
        assert br.wait_caught_up(10)
        srv.close()
        broker.fill("t", 100, "fixed_f32", size=8, records_per_batch=10)  # produced while it is down
        time.sleep(0.3)
        assert br.errors > 0 and br.running
        srv = KafkaWireServer(broker, port=port).start()
        assert wait_for(lambda: all(s["fetch_offset"] == 200 for s in br.stats()))
        for p in range(2):
            assert log_bytes(br.local, "t", p) == log_bytes(broker, "t", p)
        br.local.commit("g", {TopicPartition("t", 0): 150})
        assert wait_for(lambda: broker.committed("g", "t", 0) == 150)
    finally:
        br.close()
        srv.close()


def test_stopping_a_bridge_does_not_wait_out_a_hung_broker(broker, server):
    broker.create_topic("t", 1)
    broker.fill("t", 10, "fixed_f32", size=8)
    br = bridge(server, request_timeout_ms=30000)
    assert br.wait_caught_up(10)
    server.stall_s = 20.0  # every fetch now hangs in the broker
    time.sleep(0.3)
    t0 = time.monotonic()
    br.close(flush=False)
    assert time.monotonic() - t0 < 3.0
    server.stall_s = 0.0


# ---------------------------------------------------------------- the native (C++) wire server

def test_native_server_protocol_and_byte_identical_replica(broker):
    from torchkafka_amd.broker import NativeWireServer

    broker.create_topic("t", 3)
    broker.fill("t", 500, "fixed_f32", size=32, records_per_batch=50)
    with NativeWireServer(broker) as srv:
        c = core().WireClient(srv.address)
        assert c.metadata("t")[0] == 0 and c.metadata("nope")[0] == 3
        assert c.list_offsets("t", [0, 1, 2], -1) == {0: 500, 1: 500, 2: 500}
        assert c.offset_commit("g", "t", {1: 42}) == {1: 0}
        assert c.offset_fetch("g", "t", [0, 1]) == {0: -1, 1: 42}
        with bridge(srv, group_id="g", max_partition_fetch_bytes=8192, fetch_max_bytes=16384) as br:
            assert br.wait_caught_up(10)
            for p in range(3):
                assert log_bytes(br.local, "t", p) == log_bytes(broker, "t", p)
            assert {s["start_offset"] for s in br.stats()} == {0, 42}
            broker.fill("t", 100, "fixed_f32", size=32, records_per_batch=50)  # long-poll wakes up
            assert br.wait_caught_up(10)
            assert br.errors == 0
        assert srv.requests > 10 and srv.bytes_sent > 3 * 500 * 128


def test_native_server_cluster_and_device_loader(broker):
    import socket as _s

    from torchkafka_amd.broker import NativeWireServer

    broker.create_topic("t", 4)
    broker.fill("t", 90, "fixed_f32", size=8, records_per_batch=15)
    socks = [_s.socket() for _ in range(2)]
    for s in socks:
        s.bind(("127.0.0.1", 0))
    ports = [s.getsockname()[1] for s in socks]
    for s in socks:
        s.close()
    cluster = [(i, "127.0.0.1", ports[i]) for i in range(2)]
    nodes = [NativeWireServer(broker, port=ports[i], node_id=i, cluster=cluster).start() for i in range(2)]
    try:
        dl = DeviceLoader(Vec8.placeholder(), 12, device="cpu", num_workers=2,
                          worker_init_fn=Vec8.init_worker("t", bootstrap_servers=nodes[1].address, group_id="nat",
                                                          auto_offset_reset="earliest", consumer_timeout_ms=400))
        seen = set()
        for x in auto_commit(dl):
            seen |= {(int(p), int(o)) for o, p in x[:, :2].tolist()}
        dl.close()
        assert seen == {(p, o) for p in range(4) for o in range(90)}
        assert broker.committed_offsets("nat", "t") == {p: 90 for p in range(4)}
        assert all(n.requests > 0 for n in nodes)
    finally:
        for n in nodes:
            n.close()



# ---------------------------------------------------------------- ring replicas

def test_ring_replica_streams_more_than_its_size(broker, server):
    """A 1 MiB ring carries a ~4 MB stream: the replicator writes over committed batches, wraps, and
    waits while the consumer holds the ring (flow control); every record arrives once, in order."""
    broker.create_topic("t", 1)
    broker.fill("t", 4000, "fixed_f32", size=256, records_per_batch=16)  # ~4.2 MB, 16.6 KB batches
    with bridge(server, group_id="g", ring_bytes=1 << 20, max_partition_fetch_bytes=128 << 10,
                fetch_max_bytes=128 << 10, fetch_max_wait_ms=5) as br:
        pidx = br.local.pidx("t", 0)
        assert br.local.native.ring_bytes(pidx) == 1 << 20
        assert wait_for(lambda: br.stats()[0]["throttled"] > 0)  # nothing committed yet: the ring fills
        assert br.stats()[0]["fetch_offset"] < 4000
        c = KafkaConsumer("t", bootstrap_servers=br.url, group_id="g", auto_offset_reset="earliest",
                          enable_auto_commit=False, consumer_timeout_ms=1000)
        got = []
        for r in c:
            v = torch.frombuffer(bytearray(r.value), dtype=torch.float32)
            assert int(v[0]) == r.offset and v[2:6].tolist() == [synth_f32(0, r.offset, j) for j in range(2, 6)]
            got.append(r.offset)
            if r.offset % 100 == 99:
                c.commit()  # frees ring space for the replicator
        c.commit()
        c.close()
        assert got == list(range(4000))
        assert br.local.native.first_batch(pidx) > 0  # batches were retired and written over
        assert br.local.beginning_offset("t", 0) > 0
        br.flush()
    assert broker.committed("g", "t", 0) == 4000


def test_ring_replica_feeds_a_device_loader(broker, server):
    broker.create_topic("t", 2)
    broker.fill("t", 3000, "fixed_f32", size=64, records_per_batch=20)  # ~800 KB per partition
    with bridge(server, group_id="gr", ring_bytes=256 << 10, max_partition_fetch_bytes=32 << 10,
                fetch_max_bytes=64 << 10, fetch_max_wait_ms=5) as br:
        dl = DeviceLoader(Vec64.placeholder(), 50, device="cpu", num_workers=2,
                          worker_init_fn=Vec64.init_worker("t", bootstrap_servers=br.url, group_id="gr",
                                                           auto_offset_reset="earliest", consumer_timeout_ms=1500))
        seen = []
        for x in auto_commit(dl):
            seen += [(int(p), int(o)) for o, p in x[:, :2].tolist()]
        dl.close()
        assert sorted(seen) == [(p, o) for p in range(2) for o in range(3000)]
        assert all(br.local.native.first_batch(br.local.pidx("t", p)) > 0 for p in range(2))
    assert broker.committed_offsets("gr", "t") == {0: 3000, 1: 3000}


def test_load_state_dict_rewinds_a_bridged_cluster(broker, server):
    """A checkpoint's offsets are the cluster's: load_state_dict commits them there and mirrors
    afresh from them, even where the replica no longer holds those records (ring written over)."""
    broker.create_topic("t", 2)
    broker.fill("t", 400, "fixed_f32", size=8, records_per_batch=20)
    kw = dict(bootstrap_servers=server.address, group_id="ck", auto_offset_reset="earliest", consumer_timeout_ms=400)
    dl = DeviceLoader(Vec8.placeholder(), 20, device="cpu", num_workers=1, worker_init_fn=Vec8.init_worker("t", **kw))
    n = sum(x.shape[0] for x in auto_commit(dl))
    dl.close()
    assert n == 800 and broker.committed_offsets("ck", "t") == {0: 400, 1: 400}
    # resume from a checkpoint taken earlier in the stream
    dl2 = DeviceLoader(Vec8.placeholder(), 20, device="cpu", num_workers=1, worker_init_fn=Vec8.init_worker("t", **kw))
    dl2.load_state_dict({"version": 1, "group_id": "ck", "offsets": {"t": {0: 100, 1: 300}}})
    assert broker.committed_offsets("ck", "t") == {0: 100, 1: 300}
    got = sorted((int(p), int(o)) for x in auto_commit(dl2) for o, p in x[:, :2].tolist())
    dl2.close()
    assert got == sorted([(0, o) for o in range(100, 400)] + [(1, o) for o in range(300, 400)])
    assert broker.committed_offsets("ck", "t") == {0: 400, 1: 400}


def test_serve_cli(broker):
    import subprocess
    import sys

    broker.create_topic("t", 2)
    broker.fill("t", 10, "fixed_f32", size=8)
    p = subprocess.Popen([sys.executable, "-m", "torchkafka_amd.broker.serve", broker.url, "--port", "0"],
                         stdout=subprocess.PIPE, text=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        line = p.stdout.readline().strip()
        assert line.startswith("serving ")
        assert core().WireClient(line.rsplit(" ", 1)[1]).list_offsets("t", [0, 1], -1) == {0: 10, 1: 10}
    finally:
        p.terminate()
        p.wait(10)


# ---- TLS and SASL/PLAIN (kafka-python's security_protocol / ssl_* / sasl_* settings)

@pytest.fixture(scope="module")
def tls_cert(tmp_path_factory):
    """A self-signed certificate for 127.0.0.1 (openssl CLI; the test is skipped without it)."""
    import shutil
    import subprocess
    if shutil.which("openssl") is None:
        pytest.skip("openssl CLI not available")
    d = tmp_path_factory.mktemp("tls")
    cert, key = str(d / "cert.pem"), str(d / "key.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", cert,
                    "-days", "1", "-subj", "/CN=127.0.0.1", "-addext", "subjectAltName=IP:127.0.0.1"],
                   check=True, capture_output=True)
    return cert, key


def secure_server(broker, tls_cert=None, users=None):
    import ssl
    ctx = None
    if tls_cert is not None:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(*tls_cert)
    return KafkaWireServer(broker, ssl_context=ctx, sasl_users=users).start()


def test_tls_replica_is_byte_identical(broker, tls_cert):
    broker.create_topic("t", 2)
    broker.fill("t", 300, "fixed_f32", size=16, records_per_batch=25)
    srv = secure_server(broker, tls_cert)
    try:
        with bridge(srv, group_id="g", security_protocol="SSL", ssl_cafile=tls_cert[0]) as br:
            assert br.wait_caught_up(10)
            for p in range(2):
                assert log_bytes(br.local, "t", p) == log_bytes(broker, "t", p)
            br.local.commit("g", {TopicPartition("t", 0): 123})
            assert wait_for(lambda: broker.committed_offsets("g", "t").get(0) == 123)
        # an untrusted certificate (no cafile -> system roots) fails the handshake
        with pytest.raises(Exception, match="(?i)ssl|certificate|NoBrokersAvailable"):
            core().WireClient(srv.address, timeout_ms=2000, security={"security_protocol": "SSL"}).metadata("t")
        # a plaintext client on a TLS listener gets nowhere
        with pytest.raises(Exception):
            core().WireClient(srv.address, timeout_ms=1000).metadata("t")
    finally:
        srv.close()


def test_sasl_plain_authenticates(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 50, "fixed_f32", size=8)
    srv = secure_server(broker, users={"alice": "s3cret"})
    try:
        sec = {"security_protocol": "SASL_PLAINTEXT", "sasl_mechanism": "PLAIN", "sasl_plain_username": "alice"}
        c = core().WireClient(srv.address, timeout_ms=2000, security=dict(sec, sasl_plain_password="s3cret"))
        assert c.list_offsets("t", [0], -1) == {0: 50}
        with pytest.raises(Exception, match="(?i)auth"):
            core().WireClient(srv.address, timeout_ms=2000,
                              security=dict(sec, sasl_plain_password="wrong")).metadata("t")
        # no credentials: the listener drops the unauthenticated request
        with pytest.raises(Exception):
            core().WireClient(srv.address, timeout_ms=1000).metadata("t")
        with bridge(srv, group_id="g", security_protocol="SASL_PLAINTEXT", sasl_mechanism="PLAIN",
                    sasl_plain_username="alice", sasl_plain_password="s3cret") as br:
            assert br.wait_caught_up(10) and br.local.end_offset("t", 0) == 50
    finally:
        srv.close()


def test_sasl_ssl_combined(broker, tls_cert):
    broker.create_topic("t", 2)
    broker.fill("t", 120, "fixed_f32", size=8, records_per_batch=10)
    srv = secure_server(broker, tls_cert, users={"bob": "pw"})
    try:
        with bridge(srv, group_id="g", security_protocol="SASL_SSL", ssl_cafile=tls_cert[0],
                    sasl_plain_username="bob", sasl_plain_password="pw") as br:
            assert br.wait_caught_up(10)
            assert all(log_bytes(br.local, "t", p) == log_bytes(broker, "t", p) for p in range(2))
    finally:
        srv.close()


def test_security_config_validates_the_mechanism():
    from torchkafka_amd.broker.bridge import security_config
    assert security_config(security_protocol="SSL", ssl_cafile=None, bootstrap_servers="x") == \
        {"security_protocol": "SSL"}
    with pytest.raises(ValueError, match="PLAIN"):
        security_config(security_protocol="SASL_SSL", sasl_mechanism="GSSAPI")


@pytest.mark.parametrize("mech", ["SCRAM-SHA-256", "SCRAM-SHA-512"])
def test_sasl_scram_authenticates(broker, tls_cert, mech):
    broker.create_topic("t", 2)
    broker.fill("t", 30, "fixed_f32", size=8)
    srv = secure_server(broker, tls_cert, users={"carol": "p,w=d"})
    try:
        sec = {"security_protocol": "SASL_SSL", "ssl_cafile": tls_cert[0], "sasl_mechanism": mech,
               "sasl_plain_username": "carol"}
        c = core().WireClient(srv.address, timeout_ms=2000, security=dict(sec, sasl_plain_password="p,w=d"))
        assert c.list_offsets("t", [0, 1], -1) == {0: 30, 1: 30}
        with pytest.raises(Exception, match="SaslAuthenticationFailed"):
            bad = dict(sec, sasl_plain_password="nope")
            core().WireClient(srv.address, timeout_ms=2000, security=bad).metadata("t")
        with bridge(srv, group_id="g", security_protocol="SASL_SSL", ssl_cafile=tls_cert[0], sasl_mechanism=mech,
                    sasl_plain_username="carol", sasl_plain_password="p,w=d") as br:
            assert br.wait_caught_up(10) and br.local.end_offset("t", 1) == 30
    finally:
        srv.close()


class _Tokens:
    """kafka-python's AbstractTokenProvider shape: token() (rotating) and extensions()."""

    def __init__(self, tokens, extensions=None):
        self.tokens, self.ext, self.calls = list(tokens), extensions, 0

    def token(self):
        self.calls += 1
        return self.tokens[min(self.calls - 1, len(self.tokens) - 1)]

    def extensions(self):
        return self.ext or {}


@pytest.mark.parametrize("profile", ["legacy", "kafka4"])
def test_sasl_oauthbearer_authenticates(broker, profile):
    """SASL/OAUTHBEARER (RFC 7628): the token comes from kafka-python's sasl_oauth_token_provider,
    extensions ride in the client message, a bad token fails the exchange, and a KafkaBridge
    refreshes the token for the connections it makes later."""
    from torchkafka_amd.broker.bridge import security_config

    broker.create_topic("t", 2)
    broker.fill("t", 40, "fixed_f32", size=8)
    srv = KafkaWireServer(broker, profile=profile, sasl_oauth_tokens={"tok-1": "svc", "tok-2": "svc"}).start()
    try:
        base = {"security_protocol": "SASL_PLAINTEXT", "sasl_mechanism": "OAUTHBEARER"}
        sec = security_config(**base, sasl_oauth_token_provider=_Tokens(["tok-1"], {"traceId": "abc"}))
        assert sec["sasl_oauth_token"] == "tok-1" and sec["sasl_oauth_extensions"] == "traceId=abc"
        c = core().WireClient(srv.address, timeout_ms=2000, security=sec)
        assert c.list_offsets("t", [0, 1], -1) == {0: 40, 1: 40}
        assert srv.oauth_log[-1] == ("tok-1", {"traceId": "abc"}, True)
        with pytest.raises(Exception, match="SaslAuthenticationFailed"):
            bad = security_config(**base, sasl_oauth_token_provider=_Tokens(["forged"]))
            core().WireClient(srv.address, timeout_ms=2000, security=bad).metadata("t")
        assert srv.oauth_log[-1][2] is False
        with pytest.raises(ValueError, match="sasl_oauth_token_provider"):
            security_config(**base)
        prov = _Tokens(["tok-1", "tok-2"])
        with bridge(srv, group_id="g", security_protocol="SASL_PLAINTEXT", sasl_mechanism="OAUTHBEARER",
                    sasl_oauth_token_provider=prov, oauth_refresh_s=0.05) as br:
            assert br.wait_caught_up(10) and br.local.end_offset("t", 1) == 40
            assert wait_for(lambda: prov.calls >= 2)  # refreshed from the bridge's Python thread
            br.local.commit("g", {TopicPartition("t", 0): 7})  # the commit client connects later
            assert wait_for(lambda: broker.committed_offsets("g", "t").get(0) == 7)
        assert {tok for tok, _, ok in srv.oauth_log if ok} >= {"tok-1"}
    finally:
        srv.close()


# ---- group membership: subscribe mode (JoinGroup / SyncGroup / Heartbeat / LeaveGroup)

def test_range_assignor_matches_kafkas():
    got = core().range_assign([("c", ["t"]), ("a", ["t", "u"]), ("b", ["t"])], {"t": 8, "u": 3})
    assert got == {"a": {"t": [0, 1, 2], "u": [0, 1, 2]}, "b": {"t": [3, 4, 5]}, "c": {"t": [6, 7]}}
    assert core().range_assign([("a", ["t"]), ("b", ["t"]), ("c", ["t"])], {"t": 2})["c"] == {"t": []}
    rr = core().range_assign([("b", ["t", "u"]), ("a", ["t"])], {"t": 5, "u": 2}, roundrobin=True)
    assert rr == {"a": {"t": [0, 2, 4]}, "b": {"t": [1, 3], "u": [0, 1]}}


def test_roundrobin_strategy_through_the_coordinator(broker, server):
    broker.create_topic("t", 5)
    broker.fill("t", 20, "fixed_f32", size=8)
    kw = dict(group_id="g", subscribe=True, partition_assignment_strategy=["roundrobin", "range"], start=False)
    bs = [bridge(server, **kw) for _ in range(2)]
    try:
        _start_all(bs)
        assert sorted(sorted(b.assignment) for b in bs) == [[0, 2, 4], [1, 3]]
    finally:
        for b in bs:
            b.close()
    with pytest.raises(Exception, match="range . roundrobin"):
        bridge(server, group_id="g", subscribe=True, partition_assignment_strategy=["sticky"])


def _start_all(bridges):
    import threading
    errs = []

    def go(b):
        try:
            b.start()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)
    ts = [threading.Thread(target=go, args=(b,)) for b in bridges]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert not errs, errs


def test_subscribe_splits_partitions_across_members(broker, server):
    broker.create_topic("t", 6)
    broker.fill("t", 200, "fixed_f32", size=8, records_per_batch=20)
    kw = dict(group_id="g", subscribe=True, heartbeat_interval_ms=100, start=False)
    bs = [bridge(server, **kw) for _ in range(2)]
    try:
        _start_all(bs)
        a, b = (sorted(x.assignment) for x in bs)
        assert sorted(a + b) == list(range(6)) and len(a) == len(b) == 3
        assert bs[0].generation == bs[1].generation >= 1 and bs[0].member_id != bs[1].member_id
        for x in bs:
            assert x.wait_caught_up(10)
            for p in x.assignment:
                assert log_bytes(x.local, "t", p) == log_bytes(broker, "t", p)
            others = set(range(6)) - set(x.assignment)
            assert all(x.local.end_offset("t", p) == 0 for p in others)
            x.local.commit("g", {TopicPartition("t", p): 150 for p in x.assignment})
        # commits carry the member's generation and reach the cluster
        assert wait_for(lambda: broker.committed_offsets("g", "t") == {p: 150 for p in range(6)})
        stale = core().WireClient(server.address).offset_commit("g", "t", {0: 1}, "", bs[0].generation - 1,
                                                               bs[0].member_id)
        assert stale == {0: 22}  # IllegalGeneration: a zombie member is fenced
        assert len(server.group_members("g")) == 2
    finally:
        for x in bs:
            x.close()
    assert server.group_members("g") == {}  # both left the group on close


def test_a_rebalance_moves_partitions_in_process(broker, server):
    """A second member joins: the first one gives up half of the topic without stopping -- the
    partitions it keeps carry on, the revoked ones stop fetching, and when the second member leaves
    the first one gets every partition back in the next rebalance (no session-timeout wait)."""
    broker.create_topic("t", 4)
    broker.fill("t", 40, "fixed_f32", size=8)
    kw = dict(group_id="g", subscribe=True, heartbeat_interval_ms=50, session_timeout_ms=3000)
    first = bridge(server, **kw)
    try:
        assert sorted(first.assignment) == [0, 1, 2, 3] and first.wait_caught_up(10)
        e0 = first.assignment_epoch
        first.local.commit("g", {TopicPartition("t", p): 10 for p in range(4)})
        second = bridge(server, **kw)  # `first` rejoins on its next heartbeat; the range assignor halves t
        try:
            assert wait_for(lambda: len(first.assignment) == 2, 5)
            a, b = sorted(first.assignment), sorted(second.assignment)
            assert sorted(a + b) == [0, 1, 2, 3] and second.generation == first.generation == 2
            assert first.assignment_epoch > e0 and first.rebalances == 1 and not first.fenced
            # what first consumed before the rebalance reached the cluster; second starts there
            assert broker.committed_offsets("g", "t") == {p: 10 for p in range(4)}
            assert {s["partition"]: s["start_offset"] for s in second.stats() if s["owned"]} == {p: 10 for p in b}
            assert second.wait_caught_up(10)
            # new records reach each partition's new owner only
            broker.fill("t", 5, "fixed_f32", size=8)
            assert first.wait_caught_up(10) and second.wait_caught_up(10)
            for p in a:
                assert first.local.end_offset("t", p) == 45
            for p in b:
                assert second.local.end_offset("t", p) == 45 and first.local.end_offset("t", p) == 40
            second.local.commit("g", {TopicPartition("t", p): 45 for p in b})
            assert wait_for(lambda: all(broker.committed_offsets("g", "t")[p] == 45 for p in b))
        finally:
            second.close()
        # the survivor takes every partition back within one rebalance; those it gets back restart
        # at the group's committed offset (45), not where its own replica stopped (40)
        assert wait_for(lambda: sorted(first.assignment) == [0, 1, 2, 3], 5)
        assert first.generation == 3 and first.errors == 0
        starts = {s["partition"]: s["start_offset"] for s in first.stats()}
        assert all(starts[p] == 45 for p in b)
        epochs = dict(first.assignment_epochs())
        assert all(epochs[p] > epochs[q] for p in b for q in a)
        assert first.wait_caught_up(10)
        for p in b:
            assert first.local.end_offset("t", p) == 45
            assert first.local.committed_offsets("g", "t")[p] == 45
    finally:
        first.close()


def test_a_rebalance_that_keeps_the_partitions_carries_on(broker, server):
    broker.create_topic("t", 2)
    broker.create_topic("u", 2)
    broker.fill("t", 30, "fixed_f32", size=8)
    broker.fill("u", 30, "fixed_f32", size=8)
    kw = dict(group_id="g", subscribe=True, heartbeat_interval_ms=50, session_timeout_ms=3000)
    a = bridge(server, "t", **kw)
    try:
        b = bridge(server, "u", **kw)  # another topic in the same group: a keeps all of t
        try:
            assert wait_for(lambda: a.generation == 2, 5) and a.rebalances == 1
            assert sorted(a.assignment) == [0, 1] and sorted(b.assignment) == [0, 1]
            a.local.commit("g", {TopicPartition("t", 0): 30})
            assert wait_for(lambda: broker.committed_offsets("g", "t").get(0) == 30)  # generation 2 commit
        finally:
            b.close()
    finally:
        a.close()


# ---- protocol version negotiation (ApiVersions)

def test_client_negotiates_the_highest_common_version(broker, server):
    broker.create_topic("t", 2)
    broker.fill("t", 30, "fixed_f32", size=8)
    kw = dict(group_id="g", subscribe=True, heartbeat_interval_ms=50, session_timeout_ms=3000)
    with bridge(server, **kw) as br:
        assert br.wait_caught_up(10)
        br.local.commit("g", {TopicPartition("t", 0): 30})
        assert wait_for(lambda: broker.committed_offsets("g", "t").get(0) == 30)
    seen = {k: max(v) for k, v in server.request_versions.items()}
    cv = core().client_versions()
    for key, (lo, hi) in server.versions.items():
        if key in seen and key in cv:
            assert seen[key] == min(hi, cv[key][1]), (key, seen[key])
    if server.profile == "kafka4":
        assert (seen[3], seen[1], seen[11], seen[14], seen[8], seen[9], seen[2], seen[10]) == (8, 11, 5, 3, 7, 5, 5, 2)
    else:  # the versions the client hard-coded before it negotiated
        assert (seen[3], seen[1], seen[11], seen[14], seen[8], seen[9], seen[2], seen[10]) == (1, 4, 0, 0, 2, 1, 1, 0)


def test_ancient_broker_without_api_versions(broker):
    """A broker that predates ApiVersions closes the connection on it: the client reconnects and
    uses the fixed pre-negotiation versions."""
    broker.create_topic("t", 2)
    broker.fill("t", 30, "fixed_f32", size=8, records_per_batch=10)
    with KafkaWireServer(broker, profile="ancient") as srv:
        c = core().WireClient(srv.address)
        assert c.list_offsets("t", [0, 1], -1) == {0: 30, 1: 30}
        assert c.offset_commit("g", "t", {1: 7}) == {1: 0} and c.offset_fetch("g", "t", [1]) == {1: 7}
        with bridge(srv, group_id="g") as br:
            assert br.wait_caught_up(10)
            assert log_bytes(br.local, "t", 0) == log_bytes(broker, "t", 0)
        assert 18 not in srv.request_versions or srv.requests[18] >= 1


def test_no_common_version_is_unsupported_version(broker):
    broker.create_topic("t", 1)
    future = dict(KW_PROFILES["kafka4"])
    future[3] = (12, 13)  # a broker that only speaks Metadata v12+ (flexible versions)
    with KafkaWireServer(broker, profile=future) as srv:
        c = core().WireClient(srv.address)
        with pytest.raises(Exception, match="UnsupportedVersionError"):
            c.metadata("t")


@pytest.mark.parametrize("profile", ["legacy", "kafka4", "ancient"])
def test_native_server_profiles(broker, profile):
    from torchkafka_amd.broker import NativeWireServer

    broker.create_topic("t", 2)
    broker.fill("t", 300, "fixed_f32", size=16, records_per_batch=30)
    with NativeWireServer(broker, profile=profile) as srv:
        c = core().WireClient(srv.address)
        assert c.list_offsets("t", [0, 1], -2) == {0: 0, 1: 0}
        assert c.offset_commit("g", "t", {0: 5}) == {0: 0} and c.offset_fetch("g", "t", [0, 1]) == {0: 5, 1: -1}
        with bridge(srv, group_id="g", max_partition_fetch_bytes=8192) as br:
            assert br.wait_caught_up(10) and br.errors == 0
            for p in range(2):  # partition 0 starts at the committed 5, inside the first batch
                assert log_bytes(br.local, "t", p) == log_bytes(broker, "t", p)


def test_subscribe_needs_a_group(broker, server):
    with pytest.raises(ValueError, match="group_id"):
        KafkaBridge(server.address, "t", subscribe=True)
    with pytest.raises(ValueError, match="no partitions"):
        KafkaBridge(server.address, "t", group_id="g", subscribe=True, partitions=[0])


# ---- commit="sync": batch k's OffsetCommit answered before batch k+1 is handed out

@pytest.mark.parametrize("workers,bridge_mode", [(0, "auto"), (2, "auto"), (2, False)])
def test_sync_commit_reaches_the_coordinator_before_the_next_batch(broker, server, workers, bridge_mode):
    broker.create_topic("t", 4)
    broker.fill("t", 60, "fixed_f32", size=8, records_per_batch=10)
    dl = DeviceLoader(Vec8.placeholder() if workers else Vec8("t", bootstrap_servers=server.address, group_id="s",
                                                               auto_offset_reset="earliest", consumer_timeout_ms=500,
                                                               assignment="static"),
                      12, device="cpu", num_workers=workers, bridge=bridge_mode, commit="sync",
                      worker_init_fn=Vec8.init_worker("t", bootstrap_servers=server.address, group_id="s",
                                                      auto_offset_reset="earliest", consumer_timeout_ms=500,
                                                      assignment="static") if workers else None)
    prev, n = None, 0
    for x in auto_commit(dl):
        if prev is not None:  # every record of the previous batch is committed at the cluster
            got = broker.committed_offsets("s", "t")
            for o, p in prev:
                assert got.get(p) is not None and got[p] >= o + 1, (p, o, got)
        prev = [(int(o), int(p)) for o, p in x[:, :2].tolist()]
        n += x.shape[0]
    st = dl.stats_summary()
    dl.close()
    assert n == 240 and broker.committed_offsets("s", "t") == {p: 60 for p in range(4)}
    assert st["sync_commits"] >= 240 // 12 - 1 and st["commit_failures"] == 0
