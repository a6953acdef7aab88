"""RecordBatch v2 codec, CRC32C and the JSON parser against independent Python implementations."""
import json
import random
import struct

import pytest
import torch

from torchkafka_amd.ops.native import core


# --------------------------------------------------------------------------- pure-Python reference codec
def py_crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def zz(v: int) -> int:
    return (v << 1) ^ (v >> 63)


def varint(v: int) -> bytes:
    u = zz(v) & 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while u >= 0x80:
        out.append((u & 0x7F) | 0x80)
        u >>= 7
    out.append(u)
    return bytes(out)


def py_encode_batch(base_offset, values, keys, timestamps, headers):
    base_ts = min(timestamps)
    recs = bytearray()
    for i, (v, k, ts, h) in enumerate(zip(values, keys, timestamps, headers)):
        body = bytearray(b"\x00")
        body += varint(ts - base_ts) + varint(i)
        body += varint(-1) if k is None else varint(len(k)) + k
        body += varint(-1) if v is None else varint(len(v)) + v
        h = h or []
        body += varint(len(h))
        for hk, hv in h:
            hkb = hk.encode()
            body += varint(len(hkb)) + hkb
            body += varint(-1) if hv is None else varint(len(hv)) + hv
        recs += varint(len(body)) + body
    tail = struct.pack(">hiqqqhii", 0, len(values) - 1, base_ts, max(timestamps), -1, -1, -1, len(values)) + recs
    crc = py_crc32c(tail)
    head = struct.pack(">qiibI", base_offset, len(tail) + 9, 0, 2, crc)
    return head + tail


# --------------------------------------------------------------------------- tests
def test_crc32c_known_vectors():
    c = core()
    assert c.crc32c(b"123456789") == 0xE3069283
    assert c.crc32c(b"") == 0
    assert c.crc32c(b"\x00" * 32) == 0x8A9136AA
    assert c.crc32c(bytes(range(32))) == 0x46DD794E


@pytest.mark.parametrize("n", [1, 7, 8, 383, 384, 385, 3071, 3072, 3073, 24575, 24576, 24577, 100003])
def test_crc32c_interleaved_streams_match_bitwise(n):
    rnd = random.Random(n)
    data = bytes(rnd.getrandbits(8) for _ in range(n))
    exp = py_crc32c(data) if n < 5000 else None
    got = core().crc32c(data)
    if exp is not None:
        assert got == exp
    # split invariance: crc of whole == crc recomputed on a copy with different alignment
    assert core().crc32c(b"\x00" + data)  # runs the unaligned head path
    assert core().crc32c(bytes(data)) == got


def test_encode_matches_python_reference():
    rnd = random.Random(1)
    n = 20
    values = [bytes(rnd.getrandbits(8) for _ in range(rnd.randint(0, 300))) for _ in range(n)]
    values[3] = None
    keys = [None if i % 3 else f"k{i}".encode() for i in range(n)]
    ts = [1_700_000_000_000 + rnd.randint(-50, 5000) for _ in range(n)]
    headers = [None] * n
    headers[5] = [("trace", b"abc"), ("empty", None)]
    got = core().encode_batch(1000, values, keys, ts, headers)
    exp = py_encode_batch(1000, values, keys, ts, headers)
    assert got == exp


def test_decode_roundtrip_and_fields():
    values = [b"a" * 10, None, b"", b"xyz"]
    keys = [b"k0", None, b"k2", b""]
    ts = [5, 9, 7, 6]
    headers = [[("h", b"v")], None, [("x", None)], None]
    data = core().encode_batch(42, values, keys, ts, headers)
    recs = core().decode_batches(data + core().encode_batch(46, [b"n"], [None], [1], [None]))
    assert [r[0] for r in recs] == [42, 43, 44, 45, 46]
    assert [r[1] for r in recs[:4]] == ts
    assert [r[4] for r in recs[:4]] == values
    assert [r[3] for r in recs[:4]] == keys
    assert recs[0][5] == [("h", b"v")] and recs[2][5] == [("x", None)]
    # serialized sizes as kafka-python reports them
    assert recs[1][7] == -1 and recs[1][8] == -1 and recs[0][9] == 2 and recs[1][9] == -1


def test_crc_corruption_detected():
    data = bytearray(core().encode_batch(0, [b"hello world"], [None], [0], [None]))
    data[-3] ^= 0x40
    with pytest.raises(core().CorruptRecordException):
        core().decode_batches(bytes(data))
    assert core().decode_batches(bytes(data), check_crcs=False)  # decodes when not checking


@pytest.mark.parametrize("text", [
    "[1, 2.5, -3.25e2, 0.1, 1e-7, 123456789012345678901234, -0.0]",
    "[]", "  [ 7 ]  ", "[NaN, Infinity, -Infinity]", "[3.4028235e38, 1e39, 1.17549435e-38, 4e-320]",
    "[0.30000000000000004, 2.2250738585072014e-308, 9007199254740993]",
])
def test_json_parser_matches_python(text):
    got = torch.tensor(core().parse_json_f32(text.encode()), dtype=torch.float32)
    exp = torch.tensor([float(x) for x in json.loads(text)], dtype=torch.float32)
    assert got.shape == exp.shape
    assert torch.equal(torch.isnan(got), torch.isnan(exp))
    assert torch.equal(got.nan_to_num(), exp.nan_to_num())
    assert core().json_array_len(text.encode()) == len(json.loads(text))


def test_json_parser_random_numbers():
    rnd = random.Random(7)
    vals = [rnd.uniform(-1e6, 1e6) * 10 ** rnd.randint(-20, 20) for _ in range(2000)]
    text = json.dumps(vals)
    got = torch.tensor(core().parse_json_f32(text.encode()), dtype=torch.float32)
    exp = torch.tensor(json.loads(text), dtype=torch.float64).to(torch.float32)
    assert torch.equal(got, exp)


@pytest.mark.parametrize("bad", ["[1,]", "[1 2]", "{\"a\": 1}", "[[1]]", "[\"1\"]", "[1", "1, 2", "[1.]", "[-]"])
def test_json_parser_rejects(bad):
    with pytest.raises(ValueError):
        core().parse_json_f32(bad.encode())


def test_crc32c_methods_agree():
    """Table, 3-stream crc32 instruction and AVX-512 VPCLMULQDQ folding give the same CRC32C."""
    import random

    c = core()
    rnd = random.Random(11)
    methods = [0] + ([1] if c.crc32c_hw() else []) + ([2] if c.crc32c_fold() else [])
    for n in [256, 257, 300, 511, 512, 513, 1024 + 3, 4096, 65536 + 17, 200_003]:
        for _ in range(3):
            d = rnd.randbytes(n)
            want = py_crc32c(d) if n <= 4096 else c.crc32c_method(0, d)
            got = {m: c.crc32c_method(m, d) for m in methods}
            assert set(got.values()) == {want}, (n, got, want)
            assert c.crc32c(d) == want
