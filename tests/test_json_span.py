"""Device JSON-parse and var-len slots (kPackJsonSpan / kPackVarSpan, csrc/core/span.h) on the CPU.

The gfx950 kernel is checked on the GPU (tests/test_gpu_json_span.py).  Here a worker's JSON span
fill must describe exactly the rows the host packer (PACK_JSON_F32: the worker parses every
number) takes -- same watermarks, same row count, same element counts, texts at the recorded log
positions that ``json.loads`` to the host-parsed values, worker-parsed rows for the texts that
are not "simple" -- and its segments must keep every row text whole, cover every CRC-verified
RecordBatch to its end, and chain to the header CRC.
The same holds for VarLen rows (token ids etc.): the span fill must describe exactly the rows of
the host CSR packer, values at the recorded positions, long values copied by the worker.
Reference: ``json.loads(record.value)`` in ``_process`` (README.md:54,74), kafka_dataset.py:156-162.
"""
import json
import os
import random

import numpy as np
import pytest

from torchkafka_amd.ops.native import core


def _rows(rnd, n, lo=1, hi=40, odd_every=0, nulls_every=0):
    out = []
    for i in range(n):
        if nulls_every and i % nulls_every == 3:
            out.append(None)
            continue
        k = rnd.randint(lo, hi)
        vals = [round(rnd.uniform(-1000, 1000), rnd.randint(0, 4)) for _ in range(k)]
        if odd_every and i % odd_every == 1:
            # not simple: an exponent (the worker parses it) -- or a long token
            txt = "[" + ", ".join(["1.5e3"] + [repr(v) for v in vals]) + "]"
        else:
            txt = "[" + ",".join(repr(v) for v in vals) + "]"
        out.append(txt.encode())
    return out


def _fill(broker, jspan, bs, values_per_part, rpb, *, min_len=0, max_len=-1, truncate=True, slots=10,
          check_crcs=True):
    c = core()
    topic = f"j{random.randrange(1 << 30)}"
    parts = len(values_per_part)
    broker.create_topic(topic, parts)
    for p, vals in enumerate(values_per_part):
        for i in range(0, len(vals), rpb):
            broker.produce(topic, vals[i:i + rpb], partition=p)
    t0 = broker.topic(topic)[2]
    name = f"/tkjspan-{os.getpid()}-{random.randrange(1 << 30)}"
    ring = c.Ring.create(name, 1, 2, 8 << 20)
    f = c.Fetcher(broker.native, check_crcs)
    f.assign(list(range(t0, t0 + parts)), [0] * parts)
    kind = c.PACK_JSON_TEXT if jspan else c.PACK_JSON_F32
    out = []
    try:
        for i in range(slots):
            g = i % 2
            assert ring.worker_acquire(0, g, 1000)
            rows, _sc, timed_out, _sh = f.fill_slot(ring, g, kind, 4, 0, min_len, max_len, truncate, False, bs, 50,
                                                    False, jspan)
            info = ring.slot_info(g)
            pay = bytes(ring.payload_view(g)[:info["payload_bytes"]])
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


def _host_rows(info, pay):
    n = info["n_rows"]
    offs = np.frombuffer(pay[:4 * (n + 1)], dtype=np.int32)
    vals = np.frombuffer(pay[info["values_offset"]:info["values_offset"] + 4 * int(offs[-1])], dtype=np.float32)
    return [vals[offs[r]:offs[r + 1]] for r in range(n)]


def _decode_jspan(broker, info, pay, segs, trunc):
    """numpy mirror of json_span.hip: each row parsed from its segment's bytes, CRCs chained."""
    c = core()
    n = info["n_rows"]
    tab = np.frombuffer(pay[:16 * n], dtype=np.dtype([("pos", "<u8"), ("tlen", "<i4"), ("count", "<i4")]))
    got = [None] * n
    chains = {}
    for pos, ln, pidx, flags, crc, r0, r1 in segs:
        assert r1 - r0 <= c.JSON_SPAN_MAX_SEG_ROWS
        if flags & c.SEG_HOST_ROWS:
            assert ln == 0
            for r in range(r0, r1):
                assert tab[r]["tlen"] < 0, "a host-rows segment lists a device row"
                k = int(tab[r]["count"]) if trunc < 0 else min(int(tab[r]["count"]), trunc)
                o = int(tab[r]["pos"])
                assert got[r] is None
                got[r] = np.frombuffer(pay[o:o + 4 * k], dtype=np.float32)
            continue
        assert 0 < ln <= c.SPAN_SEG_MAX
        data = broker.native.read_log(pidx, pos, ln)
        for r in range(r0, r1):
            if tab[r]["tlen"] < 0:
                continue
            p0, tl = int(tab[r]["pos"]), int(tab[r]["tlen"])
            assert pos <= p0 and p0 + tl <= pos + ln, "a row text is cut by its segment"
            vals = json.loads(data[p0 - pos:p0 + tl - pos])
            assert len(vals) == tab[r]["count"] or tab[r]["count"] == c.JSON_COUNT_ON_DEVICE
            k = len(vals) if trunc < 0 else min(len(vals), trunc)
            assert got[r] is None, "a row is listed by two segments"
            got[r] = np.array([float(v) for v in vals[:k]], dtype=np.float32)
        if flags & 4:  # kSegCrc
            first = bool(flags & 1)
            c0 = 21 if first else 0
            part = c.crc32c_span_emulate(data, c0, ln, first)
            if first:
                chains[pidx] = (0, crc)
            acc, want = chains[pidx]
            chains[pidx] = (c.crc32c_shift_raw(acc, ln - c0) ^ part, want)
            if flags & 2:
                assert chains[pidx][0] ^ 0xFFFFFFFF == want, "RecordBatch CRC mismatch"
                del chains[pidx]
    assert not chains, "a verified RecordBatch was not covered to its end"
    assert all(g is not None for g in got), "a row is in no segment"
    return got


@pytest.mark.parametrize("bs,rpb,odd,nulls,lens", [
    (64, 16, 0, 0, (1, 40)),       # small batches, RecordBatches split across slots
    (100, 64, 5, 0, (1, 40)),      # every 5th row not simple: worker-parsed
    (256, 7, 0, 9, (0, 30)),       # tombstones and empty arrays
    (32, 512, 3, 0, (200, 600)),   # RecordBatches > 128 KiB: split between row texts, chained CRCs
    (2000, 4000, 0, 0, (1, 3)),    # > 1024 rows per RecordBatch: the row limit cuts segments
])
def test_json_span_fill_matches_host_parse(broker, bs, rpb, odd, nulls, lens):
    rnd = random.Random(bs * 7 + rpb)
    n = max(4 * bs, 600)
    vals = [_rows(rnd, n, *lens, odd_every=odd, nulls_every=nulls) for _ in range(2)]
    host = _fill(broker, False, bs, vals, rpb)
    span = _fill(broker, True, bs, vals, rpb)
    assert len(host) == len(span)
    for (hr, hi, hw, hp, _), (sr, si, sw, sp, segs) in zip(host, span):
        assert hr == sr and hw == sw
        if sr == 0:
            continue
        assert si["kind"] == core().PACK_JSON_SPAN and si["n_segs"] == len(segs)
        assert si["max_row_len"] == hi["max_row_len"] and si["total_elems"] == hi["total_elems"]
        ref = _host_rows(hi, hp)
        got = _decode_jspan(broker, si, sp, segs, si["trunc_len"])
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b)
        if odd:
            assert any(s[3] & core().SEG_HOST_ROWS for s in segs)


def test_json_span_filters_like_host(broker):
    rnd = random.Random(5)
    vals = [_rows(rnd, 900, 0, 50, odd_every=4) for _ in range(3)]
    for min_len, max_len, trunc in [(10, -1, True), (0, 20, True), (5, 25, False)]:
        host = _fill(broker, False, 128, vals, 32, min_len=min_len, max_len=max_len, truncate=trunc, slots=6)
        span = _fill(broker, True, 128, vals, 32, min_len=min_len, max_len=max_len, truncate=trunc, slots=6)
        for (hr, hi, hw, hp, _), (sr, si, sw, sp, segs) in zip(host, span):
            assert hr == sr and hw == sw and si["max_row_len"] == hi["max_row_len"]
            assert si["trunc_len"] == max_len
            got = _decode_jspan(broker, si, sp, segs, si["trunc_len"])
            for a, b in zip(got, _host_rows(hi, hp)):
                np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("bs,rpb,odd,nulls,lens,max_len", [
    (100, 64, 5, 0, (1, 40), -1),
    (256, 7, 0, 9, (0, 30), 12),      # tombstones, empty arrays, truncation
    (32, 512, 3, 0, (200, 600), -1),  # RecordBatches > 128 KiB
])
def test_json_span_device_count_walks_headers_only(broker, bs, rpb, odd, nulls, lens, max_len):
    """tuning.json_count (span mode SPAN_JSON_DEV_COUNT): the worker reads no text -- every row is
    left to the device (count JSON_COUNT_ON_DEVICE, its text in the log), the slot is flagged
    SLOT_DEV_COUNT and max_row_len is the text-length bound -- over exactly the rows and
    watermarks of the host packer, whose values the texts still decode to."""
    c = core()
    rnd = random.Random(bs * 13 + rpb)
    n = max(4 * bs, 600)
    vals = [_rows(rnd, n, *lens, odd_every=odd, nulls_every=nulls) for _ in range(2)]
    host = _fill(broker, False, bs, vals, rpb, max_len=max_len)
    dev = _fill(broker, c.SPAN_JSON_DEV_COUNT, bs, vals, rpb, max_len=max_len)
    assert len(host) == len(dev)
    for (hr, hi, hw, hp, _), (sr, si, sw, sp, segs) in zip(host, dev):
        assert hr == sr and hw == sw
        if sr == 0:
            continue
        assert si["flags"] & c.SLOT_DEV_COUNT and si["kind"] == c.PACK_JSON_SPAN
        tab = np.frombuffer(sp[:16 * sr], dtype=np.dtype([("pos", "<u8"), ("tlen", "<i4"), ("count", "<i4")]))
        assert (tab["count"] == c.JSON_COUNT_ON_DEVICE).all() and (tab["tlen"] >= 0).all()
        bound = tab["tlen"] // 2 if max_len < 0 else np.minimum(tab["tlen"] // 2, max_len)
        assert si["max_row_len"] == int(bound.max()) >= hi["max_row_len"]
        got = _decode_jspan(broker, si, sp, segs, si["trunc_len"])
        for a, b in zip(got, _host_rows(hi, hp)):
            np.testing.assert_array_equal(a, b)


def test_json_span_device_count_refuses_dropping_filters(broker):
    c = core()
    vals = [[b"[1,2,3]"] * 50]
    for min_len, max_len, trunc in [(2, -1, True), (0, 2, False)]:
        with pytest.raises(ValueError, match="cannot drop rows"):
            _fill(broker, c.SPAN_JSON_DEV_COUNT, 16, vals, 8, min_len=min_len, max_len=max_len, truncate=trunc,
                  slots=1)


def test_json_span_without_crc_checks_covers_only_texts(broker):
    rnd = random.Random(11)
    vals = [_rows(rnd, 800, 5, 30)]
    span = _fill(broker, True, 200, vals, 64, check_crcs=False, slots=3)
    for sr, si, _sw, sp, segs in span:
        assert sr and all(s[3] == 0 for s in segs)
        _decode_jspan(broker, si, sp, segs, -1)


# ------------------------------------------------------------------ kPackVarSpan (VarLen)
def _var_values(rnd, n, lo, hi, esize=4, nulls_every=0, long_every=0):
    import struct
    out = []
    for i in range(n):
        if nulls_every and i % nulls_every == 3:
            out.append(None)
            continue
        k = rnd.randint(lo, hi)
        if long_every and i % long_every == 2:
            k = (core().VAR_SPAN_ROW_MAX // esize) + rnd.randint(1, 500)  # longer than a segment: worker copy
        fmt = {1: "B", 2: "h", 4: "i", 8: "q"}[esize]
        lim = (1 << (8 * esize - 1)) - 1 if esize > 1 else 255
        out.append(struct.pack(f"<{k}{fmt}", *[rnd.randint(0 if esize == 1 else -lim, lim) for _ in range(k)]))
    return out


def _fill_var(broker, vspan, bs, values, rpb, esize, *, min_len=0, max_len=-1, truncate=True, slots=8):
    c = core()
    topic = f"v{random.randrange(1 << 30)}"
    broker.create_topic(topic, len(values))
    for p, vals in enumerate(values):
        for i in range(0, len(vals), rpb):
            broker.produce(topic, vals[i:i + rpb], partition=p)
    t0 = broker.topic(topic)[2]
    ring = c.Ring.create(f"/tkvspan-{os.getpid()}-{random.randrange(1 << 30)}", 1, 2, 32 << 20)
    f = c.Fetcher(broker.native, True)
    f.assign(list(range(t0, t0 + len(values))), [0] * len(values))
    out = []
    try:
        for i in range(slots):
            g = i % 2
            assert ring.worker_acquire(0, g, 1000)
            rows, _sc, timed_out, _sh = f.fill_slot(ring, g, c.PACK_VARLEN, esize, 0, min_len, max_len, truncate,
                                                    False, bs, 50, False, vspan)
            info = ring.slot_info(g)
            pay = bytes(ring.payload_view(g)[:info["payload_bytes"]])
            out.append((rows, info, [(p - t0, a, b, n) for p, a, b, n in ring.watermarks(g)], pay,
                        ring.span_segments(g)))
            ring.worker_publish(g)
            assert ring.main_acquire(100) == g
            ring.main_release(g)
            if timed_out:
                break
    finally:
        ring.shutdown()
        ring.unlink()
    return out


def _decode_var(broker, info, pay, segs, esize, trunc):
    c = core()
    dt = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[esize]
    n = info["n_rows"]
    tab = np.frombuffer(pay[:16 * n], dtype=np.dtype([("pos", "<u8"), ("tlen", "<i4"), ("count", "<i4")]))
    got = [None] * n
    for pos, ln, pidx, flags, _crc, r0, r1 in segs:
        if flags & c.SEG_HOST_ROWS:
            for r in range(r0, r1):
                assert tab[r]["tlen"] < 0
                k = int(tab[r]["count"]) if trunc < 0 else min(int(tab[r]["count"]), trunc)
                got[r] = np.frombuffer(pay[int(tab[r]["pos"]):int(tab[r]["pos"]) + k * esize], dtype=dt)
            continue
        data = broker.native.read_log(pidx, pos, ln)
        for r in range(r0, r1):
            if tab[r]["tlen"] < 0:
                continue
            p0, tl = int(tab[r]["pos"]), int(tab[r]["tlen"])
            assert pos <= p0 and p0 + tl <= pos + ln and tl == int(tab[r]["count"]) * esize
            k = int(tab[r]["count"]) if trunc < 0 else min(int(tab[r]["count"]), trunc)
            assert got[r] is None
            got[r] = np.frombuffer(data[p0 - pos:p0 - pos + k * esize], dtype=dt)
    assert all(g is not None for g in got)
    return got


@pytest.mark.parametrize("esize,bs,rpb,lens,nulls,long_every,filt", [
    (4, 64, 16, (0, 300), 0, 0, (0, -1, True)),        # token ids, batch boundaries inside RecordBatches
    (4, 32, 64, (1, 50), 7, 13, (0, -1, True)),        # tombstones + values longer than a segment
    (2, 100, 5, (0, 40), 0, 0, (3, 20, True)),         # min_len / truncation
    (1, 50, 9, (0, 70), 5, 0, (2, 30, False)),         # max_len without truncation: skipped
    (8, 2000, 3000, (1, 2), 0, 0, (0, -1, True)),      # > 1024 rows per RecordBatch
])
def test_var_span_fill_matches_host_pack(broker, esize, bs, rpb, lens, nulls, long_every, filt):
    rnd = random.Random(esize * 100 + bs)
    n = max(3 * bs, 400)
    vals = [_var_values(rnd, n, *lens, esize=esize, nulls_every=nulls, long_every=long_every) for _ in range(2)]
    min_len, max_len, trunc = filt
    host = _fill_var(broker, False, bs, vals, rpb, esize, min_len=min_len, max_len=max_len, truncate=trunc)
    span = _fill_var(broker, True, bs, vals, rpb, esize, min_len=min_len, max_len=max_len, truncate=trunc)
    assert len(host) == len(span)
    dt = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[esize]
    for (hr, hi, hw, hp, _), (sr, si, sw, sp, segs) in zip(host, span):
        assert hr == sr and hw == sw
        if sr == 0:
            continue
        assert si["kind"] == core().PACK_VAR_SPAN
        assert si["max_row_len"] == hi["max_row_len"] and si["total_elems"] == hi["total_elems"]
        offs = np.frombuffer(hp[:4 * (hr + 1)], dtype=np.int32)
        hv = np.frombuffer(hp[hi["values_offset"]:hi["values_offset"] + esize * int(offs[-1])], dtype=dt)
        got = _decode_var(broker, si, sp, segs, esize, si["trunc_len"])
        for r in range(hr):
            np.testing.assert_array_equal(got[r], hv[offs[r]:offs[r + 1]])
