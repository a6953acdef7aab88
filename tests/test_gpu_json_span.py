"""gfx950 JSON parse straight from the pinned broker logs (DeviceLoader decode='device' with a
JsonArray schema, csrc/hip/json_span.hip) on the GPU.

Every case is compared bit for bit with json.loads + torch casts (the reference's
``json.loads(record.value)`` in ``_process``, README.md:54,74) and with the other two JSON paths
(decode='host': workers frame + copy the text for json_parse.hip; json_parse='host': workers parse).
"""
import json
import os
import random

import pytest
import torch

pytestmark = pytest.mark.gpu


def _dataset(schema):
    from torchkafka_amd import KafkaDataset

    class DS(KafkaDataset):
        pass

    DS.schema = schema
    return DS


def _bits(t: torch.Tensor) -> torch.Tensor:
    """Bit patterns, with every NaN as one pattern: torch's own CPU casts do not agree on NaN bits
    (the vectorised f32 -> bf16 cast gives 0xFFFF, the scalar one 0x7FC0), so only NaN-ness is pinned."""
    bits = t.view({1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[t.element_size()])
    if t.is_floating_point():
        nan = torch.isnan(t.float())
        if bool(nan.any()):
            bits = torch.where(nan, torch.full_like(bits, 0x7F), bits)
    return bits


def _texts(rng, n, lo, hi, odd_every=0, nulls_every=0, bad_at=None):
    out = []
    for i in range(n):
        if nulls_every and i % nulls_every == 2:
            out.append(None)
            continue
        k = rng.randint(lo, hi)
        vals = [round(rng.uniform(-1e4, 1e4), rng.randint(0, 6)) for _ in range(k)]
        if rng.random() < 0.1:
            vals = [int(v) for v in vals]
        sep = ", " if rng.random() < 0.5 else ","
        txt = "[" + sep.join(repr(v) for v in vals) + "]"
        if odd_every and i % odd_every == 1:
            txt = "[2.5e-3" + ("," if vals else "") + txt[1:]  # an exponent: the worker parses the row
        if bad_at is not None and i == bad_at:
            txt = "[1,,2]"  # passes the workers' character scan, fails the device grammar
        out.append(txt.encode())
    return out


def _produce(broker, topic, parts, texts_of, rpb):
    broker.create_topic(topic, parts)
    for p in range(parts):
        tx = texts_of(p)
        for i in range(0, len(tx), rpb):
            broker.produce(topic, tx[i:i + rpb], partition=p, keys=[b"k" * (i % 5)] * len(tx[i:i + rpb]))


def _run(broker, topic, DS, bs, group, *, decode="auto", json_parse="auto", **kw):
    from torchkafka_amd import DeviceLoader, auto_commit

    dl = DeviceLoader(DS.placeholder(), bs, device="cuda:0", decode=decode, json_parse=json_parse, in_order=True,
                      worker_init_fn=DS.init_worker(topic, bootstrap_servers=broker.url, group_id=group,
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300), **kw)
    outs = [tuple(t.clone() for t in b) for b in auto_commit(dl)]
    torch.cuda.synchronize()
    return outs, dl


def _expected(texts, bs, dtype, max_len=None, min_len=0, pad=0.0, pad_multiple=8):
    rows = []
    for t in texts:
        if t is None:
            continue
        v = [float(x) for x in json.loads(t)]
        if len(v) < min_len:
            continue
        rows.append(v if max_len is None else v[:max_len])
    out = []
    for i in range(0, len(rows), bs):
        chunk = rows[i:i + bs]
        L = max((len(r) for r in chunk), default=0)
        L = (L + pad_multiple - 1) // pad_multiple * pad_multiple  # DeviceLoader's default pad_multiple
        x = torch.full((len(chunk), L), pad, dtype=torch.float32)
        for j, r in enumerate(chunk):
            if r:
                x[j, :len(r)] = torch.tensor(r, dtype=torch.float64).to(torch.float32)
        out.append((x.to(dtype), torch.tensor([len(r) for r in chunk])))
    return out


@pytest.mark.parametrize("dtype,bs,rpb,lens,odd,nulls,workers", [
    (torch.float32, 64, 16, (0, 40), 0, 0, 1),       # batch boundaries inside RecordBatches
    (torch.bfloat16, 256, 64, (16, 256), 0, 0, 1),   # BASELINE config 4's shape
    (torch.float16, 50, 7, (0, 30), 4, 6, 1),        # worker-parsed rows and tombstones
    (torch.float8_e4m3fn, 32, 9, (1, 20), 0, 0, 1),
    (torch.float32, 16, 200, (150, 400), 3, 0, 1),   # RecordBatches > 128 KiB: chained CRCs, cut rows
])
def test_json_span_matches_json_loads(broker, dtype, bs, rpb, lens, odd, nulls, workers):
    rng = random.Random(bs * 31 + rpb)
    n = 4 * bs + 13
    texts = _texts(rng, n, *lens, odd_every=odd, nulls_every=nulls)
    _produce(broker, "t", 1, lambda p: texts, rpb)
    from torchkafka_amd import JsonArray

    DS = _dataset(JsonArray())
    got, dl = _run(broker, "t", DS, bs, "g-dev", dtype=dtype, num_workers=workers, coalesce=4)
    assert dl.plan.json_span and dl.plan.json_count  # the workers read headers only; the device counts
    exp = _expected(texts, bs, dtype)
    assert len(got) == len(exp)
    for (x, ln), (ex, el) in zip(got, exp):
        assert x.shape == ex.shape and x.dtype == dtype
        assert torch.equal(_bits(x.cpu()), _bits(ex)) and torch.equal(ln.cpu(), el)
    assert broker.committed_offsets("g-dev", "t") == {0: n}
    # the other JSON paths deliver the same bits: workers counting for the device parse, workers
    # framing + copying the text, workers parsing
    for decode, jp, jc in (("auto", "auto", "host"), ("host", "auto", "auto"), ("auto", "host", "auto")):
        other, dl2 = _run(broker, "t", DS, bs, f"g-{decode}-{jp}-{jc}", dtype=dtype, num_workers=workers,
                          decode=decode, json_parse=jp, json_count=jc)
        assert dl2.plan.json_span == (jc == "host") and not dl2.plan.json_count
        assert len(other) == len(got)
        for (x, ln), (y, lm) in zip(got, other):
            assert torch.equal(_bits(x), _bits(y)) and torch.equal(ln, lm)


_EDGE_TEXTS = [b"[1,2,3]", b"  [4, 5]  ", b"[]", b"[ ]", b"\n[7]\t", b"[1.5e3, 2]", b"[NaN, 1, Infinity]",
               b"[12345678901234567, 1]", b"[1234567890123456]", b"[-0.0, 0.5, -12.25]", b" [ 3 , 4 ] ",
               b"[1e-7]", b"[" + b",".join(b"%d" % i for i in range(300)) + b"]", b"[0.1,0.2,0.30000000000000004]"]


@pytest.mark.parametrize("pad_to,pad_multiple,dtype,bs,fused", [
    (None, 8, torch.float32, 16, "0"), (None, 1, torch.bfloat16, 7, "0"), (320, 8, torch.float32, 16, "0"),
    (320, 8, torch.float32, 16, "1"), (304, 1, torch.bfloat16, 7, "1")])
def test_json_device_count_edge_rows(broker, monkeypatch, pad_to, pad_multiple, dtype, bs, fused):
    """Device-counted rows (tuning.json_count): trimmed whitespace, empty arrays, exponents / NaN /
    Infinity / 17-digit tokens (not simple: parsed on the host at delivery), a 16-digit token (simple),
    widths from the device max (or a fixed pad_to, counted by the count kernel or -- fused -- by the
    parse kernel itself) -- bit for bit json.loads + torch casts."""
    from torchkafka_amd import JsonArray

    monkeypatch.setenv("TORCHKAFKA_JSON_FUSED_COUNT", fused)
    rng = random.Random(bs)
    texts = [_EDGE_TEXTS[rng.randrange(len(_EDGE_TEXTS))] for _ in range(300)]
    _produce(broker, "e", 1, lambda p: texts, 11)
    DS = _dataset(JsonArray())
    kw = dict(pad_multiple=pad_multiple, return_mask=True, pad_value=-3.0)
    if pad_to is not None:
        kw["pad_to"] = pad_to
    got, dl = _run(broker, "e", DS, bs, "g", dtype=dtype, num_workers=1, **kw)
    assert dl.plan.json_count
    ref, _ = _run(broker, "e", DS, bs, "g-host", dtype=dtype, num_workers=1, json_count="host", **kw)
    exp = _expected(texts, bs, dtype, pad=-3.0, pad_multiple=pad_multiple)
    assert len(got) == len(exp) == len(ref)
    for (x, ln, m), (ex, el), (y, lm, my) in zip(got, exp, ref):
        if pad_to is not None:
            ex = torch.nn.functional.pad(ex.float(), (0, pad_to - ex.shape[1]), value=-3.0).to(dtype)
        assert x.shape == ex.shape and torch.equal(_bits(x.cpu()), _bits(ex)) and torch.equal(ln.cpu(), el)
        assert torch.equal(_bits(x), _bits(y)) and torch.equal(m, my) and torch.equal(ln, lm)
        assert torch.equal(m.cpu(), torch.arange(x.shape[1])[None, :] < el[:, None])
    assert broker.committed_offsets("g", "e") == {0: 300}


@pytest.mark.parametrize("bad", [b"[1,,2]", b"5", b"[1, \"a\"]", b"[,]", b"{}"])
def test_json_device_count_malformed_row_raises_before_commit(broker, bad):
    from torchkafka_amd import DeviceLoader, JsonArray, auto_commit
    from torchkafka_amd.client.errors import CorruptRecordException

    texts = [b"[1, 2]"] * 100 + [bad] + [b"[3]"] * 60
    _produce(broker, "m", 1, lambda p: texts, 16)
    DS = _dataset(JsonArray())
    dl = DeviceLoader(DS.placeholder(), 32, num_workers=1, device="cuda:0",
                      worker_init_fn=DS.init_worker("m", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    assert dl.plan.json_count
    with pytest.raises(CorruptRecordException, match="not a flat numeric JSON array"):
        for _x in auto_commit(dl):
            torch.cuda.synchronize()
    committed = broker.committed_offsets("g", "m").get(0)
    assert committed is None or committed <= 96


def test_json_span_filters_pad_and_mask(broker):
    rng = random.Random(3)
    texts = _texts(rng, 700, 0, 60, odd_every=5)
    _produce(broker, "t", 2, lambda p: texts, 32)
    from torchkafka_amd import JsonArray

    DS = _dataset(JsonArray(min_len=4, max_len=25))
    got, dl = _run(broker, "t", DS, 100, "g", dtype=torch.float32, num_workers=2, pad_value=-7.0, return_mask=True,
                   pad_multiple=8)
    assert dl.plan.json_span
    n = 0
    for x, ln, m in got:
        assert x.shape[1] % 8 == 0 and x.shape[1] <= 32
        for j in range(x.shape[0]):
            k = int(ln[j])
            assert 4 <= k <= 25 and bool(m[j, :k].all()) and not bool(m[j, k:].any())
            assert bool((x[j, k:] == -7.0).all())
        n += x.shape[0]
    assert n == 2 * sum(1 for t in texts if len(json.loads(t)) >= 4)
    assert broker.committed_offsets("g", "t") == {0: 700, 1: 700}


def _corrupt(broker, pidx, pos):
    path = os.path.join(broker.native.dir, f"p{pidx:05d}.log")
    with open(path, "r+b") as f:
        f.seek(pos)
        b = f.read(1)
        f.seek(pos)
        f.write(bytes([b[0] ^ 0x01]))


def test_json_span_crc_failure_raises_before_commit(broker):
    """A flipped text byte that the workers' pre-scan still accepts ('1' <-> '0') is caught by the
    device CRC: the batch holding it is never committed."""
    from torchkafka_amd import DeviceLoader, JsonArray, auto_commit
    from torchkafka_amd.client.errors import CorruptRecordException

    rng = random.Random(9)
    texts = [("[" + ",".join(str(rng.randint(10, 99)) for _ in range(20)) + "]").encode() for _ in range(200)]
    _produce(broker, "c", 1, lambda p: texts, 10)
    pidx = broker.pidx("c", 0)
    log = broker.native.read_log(pidx, 0, broker.native.log_bytes(pidx))
    pos, k = 0, 0
    while k < 6:  # RecordBatch 6 (offsets 60..69)
        pos += 12 + int.from_bytes(log[pos + 8:pos + 12], "big")
        k += 1
    at = log.index(b",", pos + 80) + 1  # first digit of a number inside RecordBatch 6
    _corrupt(broker, pidx, at)
    DS = _dataset(JsonArray())
    dl = DeviceLoader(DS.placeholder(), 10, num_workers=1, device="cuda:0", coalesce=1,
                      worker_init_fn=DS.init_worker("c", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    assert dl.plan.json_span
    with pytest.raises(CorruptRecordException, match="offset 60 .*failed CRC check"):
        for _x in auto_commit(dl):
            torch.cuda.synchronize()
    committed = broker.committed_offsets("g", "c").get(0)
    assert committed is not None and committed <= 60


def test_json_span_grammar_error_raises_before_commit(broker):
    from torchkafka_amd import DeviceLoader, JsonArray, auto_commit
    from torchkafka_amd.client.errors import CorruptRecordException

    rng = random.Random(1)
    texts = _texts(rng, 300, 1, 10, bad_at=137)
    _produce(broker, "b", 1, lambda p: texts, 16)
    DS = _dataset(JsonArray())
    dl = DeviceLoader(DS.placeholder(), 32, num_workers=1, device="cuda:0",
                      worker_init_fn=DS.init_worker("b", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    with pytest.raises(CorruptRecordException, match="not a flat numeric JSON array"):
        for _x in auto_commit(dl):
            torch.cuda.synchronize()
    committed = broker.committed_offsets("g", "b").get(0)
    assert committed is None or committed <= 128


def test_json_span_groups_consumed_on_other_streams(broker):
    from torchkafka_amd import DeviceLoader, JsonArray, auto_commit

    rng = random.Random(5)
    texts = {p: _texts(rng, 512, 1, 50) for p in range(4)}
    _produce(broker, "t", 4, lambda p: texts[p], 32)
    DS = _dataset(JsonArray())
    dl = DeviceLoader(DS.placeholder(), 32, num_workers=2, device="cuda:0", coalesce=8, dtype=torch.float32,
                      worker_init_fn=DS.init_worker("t", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    side = [torch.cuda.Stream(), torch.cuda.Stream()]
    sums, total = [], 0
    it = iter(auto_commit(dl))
    k = 0
    while True:
        with torch.cuda.stream(side[k % 2]):
            try:
                x, ln = next(it)
            except StopIteration:
                break
            sums.append(x.double().sum())
            total += int(ln.sum())
        k += 1
    torch.cuda.synchronize()
    want = sum(sum(float(torch.tensor(float(v), dtype=torch.float32)) for v in json.loads(t))
               for p in range(4) for t in texts[p])
    assert total == sum(len(json.loads(t)) for p in range(4) for t in texts[p])
    assert abs(float(torch.stack(sums).sum()) - want) <= 1e-6 * max(1.0, abs(want)) + 1e-3
    assert broker.committed_offsets("g", "t") == {p: 512 for p in range(4)}


def test_json_span_through_hbm_mirror(broker):
    from torchkafka_amd import JsonArray, Tuning

    rng = random.Random(17)
    texts = _texts(rng, 2000, 20, 200, odd_every=7)
    _produce(broker, "t", 2, lambda p: texts, 40)
    DS = _dataset(JsonArray())
    a, _ = _run(broker, "t", DS, 128, "gz", dtype=torch.bfloat16, num_workers=2)
    b, dl = _run(broker, "t", DS, 128, "gm", dtype=torch.bfloat16, num_workers=2, h2d="dma",
                 tuning=Tuning(mirror_chunk_mib=1, mirror_chunks=2))
    assert dl.plan.json_span and dl.plan.mirror
    assert len(a) == len(b)
    for (x, ln), (y, lm) in zip(a, b):
        assert torch.equal(_bits(x), _bits(y)) and torch.equal(ln, lm)
    assert broker.committed_offsets("gm", "t") == {0: 2000, 1: 2000}
    assert dl.stats_summary()["mirror_copies"] > 0


@pytest.mark.parametrize("dtype,bs,rpb,lens,odd,nulls,pad_to,trunc", [
    (torch.bfloat16, 256, 64, (16, 256), 0, 0, 256, False),  # BASELINE config 4's shape
    (torch.float32, 50, 7, (0, 30), 4, 6, 32, False),         # worker-parsed and host-parsed rows, tombstones
    (torch.float16, 64, 16, (0, 90), 5, 0, 40, True),         # rows cut to pad_to (max_len + truncate)
])
def test_json_fused_count_with_pad_to(broker, monkeypatch, dtype, bs, rpb, lens, odd, nulls, pad_to, trunc):
    """A fixed width (pad_to): every parse block counts its own row (no json_count_kernel launch) and
    the batch's last block reports the rows left to the host -- bit for bit json.loads + torch casts,
    and the same bits as the separate count kernel (TORCHKAFKA_JSON_FUSED_COUNT=0)."""
    from torchkafka_amd import JsonArray

    rng = random.Random(bs * 7 + pad_to)
    n = 4 * bs + 9
    texts = _texts(rng, n, *lens, odd_every=odd, nulls_every=nulls)
    # device-counted rows that are not simple (exponents: the host parses them at delivery)
    texts = [t if t is None or i % 11 != 3 else b"[1.5e3, 2, -7.25e-1]" for i, t in enumerate(texts)]
    _produce(broker, "f", 1, lambda p: texts, rpb)
    DS = _dataset(JsonArray(max_len=pad_to, truncate=True) if trunc else JsonArray())
    kw = dict(dtype=dtype, num_workers=1, pad_to=pad_to, return_mask=True, pad_value=-1.0, coalesce=4)
    monkeypatch.setenv("TORCHKAFKA_JSON_FUSED_COUNT", "1")
    got, dl = _run(broker, "f", DS, bs, "g-fused", **kw)
    assert dl.plan.json_span and dl.plan.json_count
    monkeypatch.setenv("TORCHKAFKA_JSON_FUSED_COUNT", "0")
    ref, _ = _run(broker, "f", DS, bs, "g-sep", **kw)
    exp = _expected(texts, bs, dtype, max_len=pad_to if trunc else None, pad=-1.0, pad_multiple=1)
    assert len(got) == len(exp) == len(ref)
    for (x, ln, m), (ex, el), (y, lm, my) in zip(got, exp, ref):
        ex = torch.nn.functional.pad(ex.float(), (0, pad_to - ex.shape[1]), value=-1.0).to(dtype)
        assert x.shape == ex.shape == (len(el), pad_to) and x.dtype == dtype
        assert torch.equal(_bits(x.cpu()), _bits(ex)) and torch.equal(ln.cpu(), el)
        assert torch.equal(_bits(x), _bits(y)) and torch.equal(ln, lm) and torch.equal(m, my)
    assert broker.committed_offsets("g-fused", "f") == {0: n}


@pytest.mark.parametrize("bad", [b"[1,,2]", b"5", b"[1, \"a\"]", b"[,]", b"{}", b"[1 2]", b"[1.2.3]", b" [1,,2] ",
                                 b"[1234567890123456-7]"])
def test_json_fused_count_malformed_row_raises_before_commit(broker, monkeypatch, bad):
    from torchkafka_amd import DeviceLoader, JsonArray, auto_commit
    from torchkafka_amd.client.errors import CorruptRecordException

    monkeypatch.setenv("TORCHKAFKA_JSON_FUSED_COUNT", "1")

    texts = [b"[1, 2]"] * 100 + [bad] + [b"[3]"] * 60
    _produce(broker, "m", 1, lambda p: texts, 16)
    DS = _dataset(JsonArray())
    dl = DeviceLoader(DS.placeholder(), 32, num_workers=1, device="cuda:0", pad_to=8,
                      worker_init_fn=DS.init_worker("m", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    assert dl.plan.json_count
    with pytest.raises(CorruptRecordException, match="not a flat numeric JSON array"):
        for _x in auto_commit(dl):
            torch.cuda.synchronize()
    committed = broker.committed_offsets("g", "m").get(0)
    assert committed is None or committed <= 96
