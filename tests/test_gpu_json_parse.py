"""gfx950 JSON parse kernel (json_parse.hip) against Python's json.loads + torch casts.

Rows are framed exactly as the worker frames them (tk::JsonRowDesc + 32-byte-aligned
text, or host-parsed float32 for rows the pre-scan does not send to the device) and the
kernel output is compared bit for bit with ``torch.tensor(json.loads(row), float32).to(dtype)``.
"""
import json
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float8_e4m3fn: 3}


def _frame(texts, max_len=None):
    """Host-side framing of a batch (mirrors Fetcher::fill_slot for kPackJsonText)."""
    from torchkafka_amd.ops.native import core

    c = core()
    desc = np.zeros((len(texts), 4), dtype=np.int32)
    vals = bytearray()
    for i, t in enumerate(texts):
        at = (len(vals) + 31) // 32 * 32
        vals.extend(b"\0" * (at - len(vals)))
        cnt = c.json_scan_simple(t)
        if cnt >= 0:
            vals.extend(t)
            tlen = len(t)
        else:
            f = c.parse_json_f32(t)
            cnt = len(f)
            vals.extend(np.asarray(f, dtype=np.float32).tobytes())
            tlen = -1
        n_out = cnt if max_len is None else min(cnt, max_len)
        desc[i] = (at, tlen, cnt, n_out)
    vals.extend(b"\0" * (64 - len(vals) % 16))  # the kernel reads whole 16-byte chunks
    return desc, bytes(vals)


def _run(texts, dtype=torch.float32, L=None, max_len=None, pad=0.0):
    from torchkafka_amd.ops.native import hip

    desc, vals = _frame(texts, max_len)
    n_out = desc[:, 3]
    L = int(n_out.max(initial=0)) if L is None else L
    d_desc = torch.from_numpy(desc).cuda()
    d_vals = torch.frombuffer(bytearray(vals), dtype=torch.uint8).cuda()
    out = torch.full((len(texts), L), 7, dtype=dtype, device="cuda")
    lengths = torch.empty(len(texts), dtype=torch.int64, device="cuda")
    mask = torch.empty((len(texts), L), dtype=torch.bool, device="cuda")
    err = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    hip().launch_json_rows(d_desc.data_ptr(), d_vals.data_ptr(), out.data_ptr(), DT[dtype], len(texts), L, pad,
                           lengths.data_ptr(), mask.data_ptr(), err.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out.cpu(), lengths.cpu(), mask.cpu(), int(err.item()), desc


def _expected(texts, dtype, L, max_len=None, pad=0.0):
    exp = torch.full((len(texts), L), pad, dtype=torch.float32)
    for i, t in enumerate(texts):
        v = [float(x) for x in json.loads(t)]
        if max_len is not None:
            v = v[:max_len]
        v = v[:L]
        if v:
            exp[i, : len(v)] = torch.tensor(v, dtype=torch.float64).to(torch.float32)
    return exp.to(dtype)


def _bits_equal(a, b):
    if a.dtype == torch.float8_e4m3fn:
        return torch.equal(a.view(torch.uint8), b.view(torch.uint8))
    return torch.equal(a.view(torch.int16 if a.element_size() == 2 else torch.int32),
                       b.view(torch.int16 if b.element_size() == 2 else torch.int32))


def _random_number(rnd):
    k = rnd.random()
    if k < 0.3:
        return "%.2f" % rnd.uniform(-50, 51)
    if k < 0.5:
        return repr(rnd.uniform(-1e6, 1e6))[:16].rstrip(".")  # up to 16 characters
    if k < 0.6:
        return str(rnd.randint(-10 ** 15, 10 ** 16 - 1))
    if k < 0.7:
        return "-0" if rnd.random() < 0.5 else "0.0"
    if k < 0.8:
        return "%.*f" % (rnd.randint(0, 14), rnd.uniform(-1, 1))
    if k < 0.9:
        return repr(rnd.uniform(-1e30, 1e30))  # long / exponent: host-parsed row
    return rnd.choice(["1e5", "-2.5E-3", "NaN", "Infinity", "-Infinity", "123456789012345678"])


def _random_row(rnd, n):
    seps = [", ", ",", " , ", ",\n  ", ",\t"]
    sep = rnd.choice(seps)
    body = sep.join(_random_number(rnd) for _ in range(n))
    return (rnd.choice(["", " ", "\n"]) + "[" + rnd.choice(["", " "]) + body + rnd.choice(["", " \n"]) + "]").encode()


def _valid_numbers(t):
    try:
        return all(isinstance(x, (int, float)) for x in json.loads(t))
    except ValueError:
        return False


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float8_e4m3fn])
def test_json_rows_bit_exact(dtype):
    rnd = random.Random(1234)
    texts = [_random_row(rnd, rnd.choice([0, 1, 2, 5, 17, 64, 200, 700])) for _ in range(300)]
    texts = [t for t in texts if _valid_numbers(t)]
    out, lengths, mask, err, desc = _run(texts, dtype)
    assert err == -1
    L = out.shape[1]
    exp = _expected(texts, dtype, L)
    assert torch.equal(lengths, torch.from_numpy(desc[:, 3]).long())
    for i in range(len(texts)):
        n = int(lengths[i])
        assert bool(mask[i, :n].all()) and not bool(mask[i, n:].any())
        if dtype == torch.float8_e4m3fn:
            assert _bits_equal(out[i], exp[i]), texts[i][:200]
        else:
            a, b = out[i].float(), exp[i].float()
            assert torch.equal(a.nan_to_num(), b.nan_to_num()) and torch.equal(a.isnan(), b.isnan()), texts[i][:200]
    # both row kinds were exercised
    assert (desc[:, 1] >= 0).any() and (desc[:, 1] < 0).any()


def test_json_rows_long_rows_cross_windows():
    # rows of 3k-60k characters: tokens cut by the 2 KiB windows at every alignment
    rnd = random.Random(7)
    texts = []
    for n in (300, 1000, 4000, 8000):
        nums = ["%.*f" % (rnd.randint(0, 9), rnd.uniform(-1e5, 1e5)) for _ in range(n)]
        texts.append(("[" + ", ".join(nums) + "]").encode())
    texts.append(("[" + " " * 5000 + "1.5," + " " * 3000 + "2]").encode())  # whitespace spanning windows
    out, lengths, _mask, err, desc = _run(texts, torch.float32)
    assert err == -1
    assert (desc[:, 1] >= 0).all()
    exp = _expected(texts, torch.float32, out.shape[1])
    assert torch.equal(out, exp)


def test_json_rows_truncate_pad_and_wider_L():
    texts = [b"[1, 2, 3, 4, 5, 6]", b"[]", b"[-7.25]", b"[1e3, 2]"]
    out, lengths, mask, err, _ = _run(texts, torch.float32, L=8, max_len=4, pad=-1.0)
    assert err == -1
    assert lengths.tolist() == [4, 0, 1, 2]
    assert out[0].tolist() == [1, 2, 3, 4, -1, -1, -1, -1]
    assert out[1].tolist() == [-1] * 8
    assert out[2, :2].tolist() == [-7.25, -1]
    assert out[3, :3].tolist() == [1000.0, 2.0, -1]


@pytest.mark.parametrize("bad", [b"[1,,2]", b"[1.2.3]", b"[1 2]", b"[-]", b"[1-2]", b"[1.]", b"[,1]", b"[1,]",
                                 b"[.]", b"[--1]"])
def test_json_rows_grammar_errors_flag_the_row(bad):
    from torchkafka_amd.ops.native import core

    assert core().json_scan_simple(bad) >= 0  # passes the worker's character scan
    texts = [b"[1, 2]", bad, b"[3]"]
    out, _lengths, _mask, err, _ = _run(texts, torch.float32)
    assert err == 1
    assert out[0, :2].tolist() == [1.0, 2.0] and out[2, 0].item() == 3.0


def test_json_rows_fuzz_matches_host_parser_verdicts():
    """Random character-clean rows (what the worker sends to the device): the kernel accepts exactly
    the rows the host parser accepts, with identical float32 values, and flags the others."""
    from torchkafka_amd.ops.native import core

    c = core()
    rnd = random.Random(99)
    alphabet = "0123456789.-, "
    good, bad = [], []
    while len(good) < 300 or len(bad) < 60:
        k = rnd.random()
        if k < 0.5:
            body = "".join(rnd.choice(alphabet) for _ in range(rnd.randint(0, 60)))
        else:
            toks = []
            for _ in range(rnd.randint(1, 40)):
                t = "".join(rnd.choice("0123456789.-") for _ in range(rnd.randint(1, 16)))
                toks.append(t)
            body = rnd.choice([",", ", ", " , "]).join(toks)
        row = ("[" + body + "]").encode()
        if c.json_scan_simple(row) < 0:
            continue  # the worker parses it on the host
        try:
            c.parse_json_f32(row)
            ok = True
        except ValueError:
            ok = False
        (good if ok else bad).append(row)
    good, bad = good[:300], bad[:60]
    # valid rows: one launch, identical values
    out, lengths, _m, err, desc = _run(good, torch.float32)
    assert err == -1
    for i, row in enumerate(good):
        want = torch.tensor(c.parse_json_f32(row), dtype=torch.float32)
        got = out[i, : int(lengths[i])]
        assert torch.equal(got.view(torch.int32), want.view(torch.int32)), row
    # each malformed row is flagged (one launch per row, so the flagged index is unambiguous)
    for row in bad:
        _o, _l, _m, err, _d = _run([b"[1]", row], torch.float32)
        assert err == 1, row
