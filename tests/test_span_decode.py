"""Device-decode slots (kPackRecordSpan, csrc/core/span.h) on the CPU.

The gfx950 kernel is checked on the GPU (tests/test_gpu_span.py).  Here:
  * the CRC32C lane/tree algorithm the kernel runs, emulated on the host step for step, equals
    the reference CRC32C, alone and chained across segments (host combine);
  * a worker's span fill describes exactly the rows the host packer takes (same watermarks,
    same values at the row positions, RecordBatches covered whole for their CRC, segment
    bounds and row ranges consistent) -- a numpy "decode" of the slot reproduces the packed
    batch bit for bit.
Reference: the per-record loop kafka_dataset.py:156-162 and kafka-python's check_crcs.
"""
import os
import random
import struct

import numpy as np
import pytest

from torchkafka_amd.ops.native import core


def _crc32c_ref(b: bytes) -> int:
    return core().crc32c(b)


@pytest.mark.parametrize("n", [25, 61, 64, 300, 1057, 4096, 66_000, 65_536 + 21, 131_072 + 21, 140_000])
def test_lane_tree_crc_matches_crc32c(n):
    c = core()
    rnd = random.Random(n)
    buf = bytes(rnd.getrandbits(8) for _ in range(n))
    c1 = n if n - 21 <= c.SPAN_SEG_MAX else 21 + c.SPAN_SEG_MAX
    raw = c.crc32c_span_emulate(buf, 21, c1, True)
    assert raw ^ 0xFFFFFFFF == _crc32c_ref(buf[21:c1])


@pytest.mark.parametrize("parts", [2, 3, 4, 8])
@pytest.mark.parametrize("n", [61, 10_300, 20_500, 66_000, 131_072 + 21])
def test_segment_parts_combine_to_the_segment_crc(n, parts):
    """SpanLaunch::parts: P workgroups each fold a contiguous run of the segment's windows from a
    zero state, move every lane to the segment's end (lane constants, kSpanTabLaneMul) and
    xor it in (span_device.h crc_finish) -- the same raw CRC as one workgroup.  Parts with no window
    (segments shorter than P windows) contribute zero."""
    c = core()
    rnd = random.Random(n * 10 + parts)
    buf = bytes(rnd.getrandbits(8) for _ in range(n))
    c1 = min(n, 21 + c.SPAN_SEG_MAX)
    whole = c.crc32c_span_emulate(buf, 21, c1, True)
    assert c.crc32c_span_emulate(buf, 21, c1, True, parts) == whole
    assert whole ^ 0xFFFFFFFF == _crc32c_ref(buf[21:c1])


def test_lane_tree_crc_unaligned_ranges():
    c = core()
    rnd = random.Random(7)
    buf = bytes(rnd.getrandbits(8) for _ in range(5000))
    for c0, c1 in [(0, 5000), (3, 4999), (1, 2), (13, 17), (100, 100 + 260 * 3 + 1), (7, 4096 + 7)]:
        raw = c.crc32c_span_emulate(buf, c0, c1, c1 - c0 >= 4)
        if c1 - c0 >= 4:
            assert raw ^ 0xFFFFFFFF == _crc32c_ref(buf[c0:c1])
        else:  # raw CRC of a too-short range: compare with the linear (zero-init) definition
            assert raw == c.crc32c_shift_raw(0, 0) ^ _raw(buf[c0:c1])


def _raw(b: bytes) -> int:
    # zero-initialised, no final xor: crc32c(b) with init/xorout folded out
    c = core()
    full = _crc32c_ref(b)
    return full ^ 0xFFFFFFFF ^ c.crc32c_shift_raw(0xFFFFFFFF, len(b))


def test_segment_chain_combine():
    """Multi-segment RecordBatches: the device writes raw partials, the host chains them."""
    c = core()
    rnd = random.Random(3)
    buf = bytes(rnd.getrandbits(8) for _ in range(200_000))
    cuts = [0, 131_072, 150_001, 200_000]
    acc = 0
    for i in range(len(cuts) - 1):
        lo, hi = cuts[i], cuts[i + 1]
        c0 = lo + (21 if i == 0 else 0)
        part = c.crc32c_span_emulate(buf[lo:hi], c0 - lo, hi - lo, i == 0)
        acc = c.crc32c_shift_raw(acc, hi - c0) ^ part
    assert acc ^ 0xFFFFFFFF == _crc32c_ref(buf[21:])


# ------------------------------------------------------------------ span fill
def _fill(broker, span: bool, bs: int, *, size=256, per_part=3000, rpb=64, nulls=False, check_crcs=True,
          partitions=2, slots=None, key=None):
    c = core()
    topic = f"t{random.randrange(1 << 30)}"
    broker.create_topic(topic, partitions)
    if nulls:
        # every 7th value null (a tombstone: the schema's `_process -> None`)
        for p in range(partitions):
            vals = [None if o % 7 == 3 else struct.pack("<%df" % size, *([float(o)] * size)) for o in range(per_part)]
            for i in range(0, per_part, rpb):
                broker.produce(topic, vals[i:i + rpb], partition=p)
    else:
        broker.fill(topic, per_part, "fixed_f32", size=size, records_per_batch=rpb)
    t0 = broker.topic(topic)[2]
    name = f"/tkspan-{os.getpid()}-{random.randrange(1 << 30)}"
    ring = c.Ring.create(name, 1, 2, max(4 << 20, bs * size * 4 + (64 << 10)))
    f = c.Fetcher(broker.native, check_crcs)
    f.assign(list(range(t0, t0 + partitions)), [0] * partitions)
    out = []
    try:
        for i in range(slots or 8):
            g = i % 2
            assert ring.worker_acquire(0, g, 1000)
            rows, _sc, timed_out, _sh = f.fill_slot(ring, g, c.PACK_FIXED, 4, size, 0, -1, True, False, bs, 50,
                                                    False, span)
            info = ring.slot_info(g)
            pay = bytes(ring.payload_view(g)[:max(info["payload_bytes"], bs * size * 4 if not span else 0)])
            wms = [(p - t0, a, b, n) for p, a, b, n in ring.watermarks(g)]
            out.append((rows, info, wms, pay, ring.span_segments(g)))
            ring.worker_publish(g)
            assert ring.main_acquire(100) == g
            ring.main_release(g)
            if timed_out:
                break
    finally:
        ring.shutdown()
        ring.unlink()
    return out


def _decode_span(broker, info, pay, segs, size):
    """numpy mirror of span_decode.hip: rows from the log ranges + CRC of whole RecordBatches."""
    c = core()
    n = info["n_rows"]
    row_pos = np.frombuffer(pay[:8 * n], dtype=np.uint64)
    out = np.full((n, size), np.nan, dtype=np.float32)
    rb_bytes = size * 4
    chains = {}
    for k, (pos, ln, pidx, flags, crc, rb0, rb1) in enumerate(segs):
        assert 0 < ln <= c.SPAN_SEG_MAX and rb1 - rb0 <= c.SPAN_MAX_SEG_ROWS
        data = broker.native.read_log(pidx, pos, ln)
        for r in range(rb0, rb1):
            v0 = int(row_pos[r])
            lo, hi = max(v0, pos), min(v0 + rb_bytes, pos + ln)
            assert lo < hi, "a listed row must intersect its segment"
            assert (lo - v0) % 4 == 0 and (hi - v0) % 4 == 0, "segment cut inside an element"
            out[r, (lo - v0) // 4:(hi - v0) // 4] = np.frombuffer(data[lo - pos:hi - pos], dtype=np.float32)
        if flags & 4:  # kSegCrc
            first = bool(flags & 1)
            c0 = 21 if first else 0
            part = c.crc32c_span_emulate(data, c0, ln, first)
            if first:
                chains[pidx] = (0, crc)
            acc, want = chains[pidx]
            acc = c.crc32c_shift_raw(acc, ln - c0) ^ part
            chains[pidx] = (acc, want)
            if flags & 2:  # kSegCrcLast
                assert acc ^ 0xFFFFFFFF == want, "RecordBatch CRC mismatch"
                del chains[pidx]
    assert not chains, "a verified RecordBatch was not covered to its end"
    return out


@pytest.mark.parametrize("bs,rpb,size", [(256, 64, 256), (100, 64, 256), (256, 7, 64), (64, 3, 40_000),
                                         (4000, 512, 2)])
def test_span_fill_matches_host_pack(broker, bs, rpb, size):
    per_part = min(max(3 * bs, 1200), (24 << 20) // (size * 4))
    host = _fill(broker, False, bs, size=size, per_part=per_part, rpb=rpb)
    span = _fill(broker, True, bs, size=size, per_part=per_part, rpb=rpb)
    assert len(host) == len(span)
    seen_rbs = set()
    for (hr, hi, hw, hp, _), (sr, si, sw, sp, segs) in zip(host, span):
        assert hr == sr and hw == sw and si["kind"] == core().PACK_RECORD_SPAN
        assert si["n_segs"] == len(segs) and (len(segs) > 0) == (sr > 0)
        ref = np.frombuffer(hp[:hr * size * 4], dtype=np.float32).reshape(hr, size)
        got = _decode_span(broker, si, sp, segs, size)
        np.testing.assert_array_equal(got, ref)
        for s in segs:
            if s[3] & 1:
                assert (s[2], s[0]) not in seen_rbs, "a RecordBatch was CRC-verified twice"
                seen_rbs.add((s[2], s[0]))


def test_span_fill_skips_nulls_like_host(broker):
    host = _fill(broker, False, 50, size=8, per_part=400, rpb=16, nulls=True, slots=6)
    span = _fill(broker, True, 50, size=8, per_part=400, rpb=16, nulls=True, slots=6)
    for (hr, _hi, hw, hp, _), (sr, si, sw, sp, segs) in zip(host, span):
        assert hr == sr and hw == sw
        ref = np.frombuffer(hp[:hr * 32], dtype=np.float32).reshape(hr, 8)
        np.testing.assert_array_equal(_decode_span(broker, si, sp, segs, 8), ref)


def test_span_fill_without_crc_checks_reads_only_values(broker):
    span = _fill(broker, True, 256, size=256, per_part=1200, rpb=64, check_crcs=False, slots=3)
    for sr, si, _sw, sp, segs in span:
        assert all(s[3] == 0 for s in segs)
        assert sum(s[1] for s in segs) == sr * 1024 + (sr - len(segs)) * 0 + _gaps(si, sp, segs)


def _gaps(info, pay, segs):
    # record framing between consecutive values inside one segment (not value bytes)
    n = info["n_rows"]
    row_pos = np.frombuffer(pay[:8 * n], dtype=np.uint64)
    g = 0
    for pos, ln, _p, _f, _c, r0, r1 in segs:
        for r in range(r0 + 1, r1):
            g += int(row_pos[r]) - int(row_pos[r - 1]) - 1024
    return g
