"""Worker-side JSON pre-scan for the device parser (consumer.cpp json_scan_simple).

The scan decides which rows the gfx950 kernel parses: it must count elements exactly
and only accept rows whose numbers the kernel converts bit-exactly (<= 16 characters
from [0-9.-]).  The AVX2 and scalar implementations must agree byte for byte.
"""
import json
import random

from hypothesis import given, settings
from hypothesis import strategies as st

from torchkafka_amd.ops.native import core


def scan(b, simd=True):
    return core().json_scan_simple(b, simd)


def test_scan_examples():
    assert scan(b"[1, 2.5, -3]") == 3
    assert scan(b"[]") == 0 and scan(b" [ \n ] ") == 0
    assert scan(b"  [1,2]  \n") == 2
    assert scan(b"[1234567890123456]") == 1          # 16 characters: device
    assert scan(b"[12345678901234567]") == -1        # 17: host
    assert scan(b"[-123456789012345]") == 1
    for host in (b"[1e5]", b"[NaN]", b"[Infinity]", b"[1E-3]", b"[+1]", b'["1"]', b"[[1]]", b"{}", b"x", b"[1",
                 b"1]", b"[,]", b"[ , ]"):
        assert scan(host) == -1, host
    # malformed but character-clean rows go to the device, which flags them
    assert scan(b"[1,,2]") == 3 and scan(b"[1.2.3]") == 1 and scan(b"[1 2]") == 1


def test_scan_counts_match_json_for_simple_rows():
    rnd = random.Random(3)
    for _ in range(3000):
        n = rnd.randint(0, 300)
        nums = ["%.*f" % (rnd.randint(0, 6), rnd.uniform(-1e6, 1e6)) for _ in range(n)]
        s = ("[" + rnd.choice([",", ", ", " ,\n"]).join(nums) + "]").encode()
        expect = len(json.loads(s)) if all(len(x) <= 16 for x in nums) else -1
        assert scan(s) == expect
        assert scan(s, False) == expect


@settings(max_examples=3000, deadline=None)
@given(st.binary(max_size=300), st.sampled_from([b"", b" ", b"\n\t"]))
def test_scan_simd_matches_scalar_on_arbitrary_bytes(body, ws):
    for s in (b"[" + body + b"]", ws + b"[" + body + b"]" + ws, body):
        assert scan(s) == scan(s, False)


@settings(max_examples=2000, deadline=None)
@given(st.lists(st.text(alphabet="0123456789.-", min_size=0, max_size=40), max_size=40),
       st.sampled_from([",", ", ", " , ", ",\n"]))
def test_scan_simd_matches_scalar_on_token_runs(tokens, sep):
    # long runs of number characters around every 32-byte block boundary
    s = ("[" + sep.join(tokens) + "]").encode()
    assert scan(s) == scan(s, False)
    if scan(s) >= 0:
        assert all(len(t) <= 16 for t in tokens)
        assert scan(s) == (len(tokens) if any(tokens) else 0) or not all(tokens)


def test_negative_zero_follows_python_float():
    import math

    for text in (b"[-0]", b"[-0.0]", b"[-0e0]", b"[-00]", b"[-0.000]"):
        got = core().parse_json_f32(text)
        exp = [float(x) for x in json.loads(text)] if text != b"[-00]" else [0.0]
        assert [math.copysign(1.0, v) for v in got] == [math.copysign(1.0, v) for v in exp], text


@settings(max_examples=3000, deadline=None)
@given(st.binary(max_size=300), st.sampled_from([b"", b" ", b"\n\t  "]),
       st.lists(st.text(alphabet="0123456789.-", min_size=1, max_size=20), max_size=30))
def test_fused_scan_copy_matches_scan(body, ws, tokens):
    # the worker's hot path (scan fused with the streaming copy) == the reference scan, and copies
    c = core()
    for s in (ws + b"[" + body + b"]" + ws, body, ws + ("[" + ", ".join(tokens) + "]").encode() + ws):
        cnt, same = c.json_scan_copy(s)
        assert same
        assert cnt == scan(s, False), s


@settings(max_examples=3000, deadline=None)
@given(st.binary(max_size=400), st.sampled_from([b"", b" ", b"\n\t  "]),
       st.lists(st.text(alphabet="0123456789.-", min_size=1, max_size=20), max_size=60))
def test_inplace_scan_matches_scan(body, ws, tokens):
    # the device-parse-from-the-log worker scan (64-byte blocks, garbage past the row) == the reference scan
    c = core()
    for s in (ws + b"[" + body + b"]" + ws, body, ws + ("[" + ", ".join(tokens) + "]").encode() + ws):
        for variant in (0, 1, 2, 3):
            assert c.json_scan_inplace(s, variant)[0] == scan(s, False), (variant, s)


def test_inplace_scan_long_rows_and_block_edges():
    c = core()
    rnd = random.Random(8)
    for n in list(range(0, 200)) + [1000, 5000]:
        nums = ["%.*f" % (rnd.randint(0, 4), rnd.uniform(-1e5, 1e5)) for _ in range(n)]
        s = ("[" + ",".join(nums) + "]").encode()
        for variant in (0, 1):
            assert c.json_scan_inplace(s, variant)[0] == scan(s, False) == \
                (len(nums) if all(len(x) <= 16 for x in nums) else -1)
    # a 17-character run straddling a 64-byte block boundary
    for pad in range(40, 70):
        s = b"[" + b"1," * (pad // 2) + b"12345678901234567" + b"]"
        for variant in (0, 1):
            assert c.json_scan_inplace(s, variant)[0] == -1 == scan(s, False)
