"""Property-based tests (hypothesis) for the host-side codecs and the sharding map.

The native implementations are checked against the independent pure-Python ones
in ``test_codec.py`` over generated inputs rather than hand-picked cases.
"""
import json
import math

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from torchkafka_amd.ops.native import core
from torchkafka_amd.parallel.sharding import shard_owner, shard_partitions

from test_codec import py_crc32c, py_encode_batch

SETTINGS = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])

_bytes_or_none = st.one_of(st.none(), st.binary(max_size=200))
_header = st.tuples(st.text(max_size=8), st.one_of(st.none(), st.binary(max_size=16)))
_record = st.tuples(_bytes_or_none, _bytes_or_none, st.integers(0, 2 ** 41),
                    st.one_of(st.none(), st.lists(_header, min_size=1, max_size=3)))


@SETTINGS
@given(st.binary(max_size=3000))
def test_crc32c_matches_bitwise(data):
    assert core().crc32c(data) == py_crc32c(data)


@SETTINGS
@given(st.binary(max_size=600), st.binary(max_size=600))
def test_crc32c_extends(a, b):
    # CRC of a concatenation is independent of how the input was chunked by the interleaved kernel
    assert core().crc32c(a + b) == py_crc32c(a + b)


@SETTINGS
@given(st.integers(0, 2 ** 40), st.lists(_record, min_size=1, max_size=12))
def test_encode_decode_roundtrip(base, recs):
    values, keys, ts, headers = (list(x) for x in zip(*recs))
    enc = core().encode_batch(base, values, keys, ts, headers)
    assert enc == py_encode_batch(base, values, keys, ts, headers)
    dec = core().decode_batches(enc)
    assert [r[0] for r in dec] == list(range(base, base + len(recs)))
    assert [r[1] for r in dec] == ts
    assert [r[3] for r in dec] == keys
    assert [r[4] for r in dec] == values
    assert [r[5] or None for r in dec] == [h or None for h in headers]


_f = st.one_of(st.floats(allow_nan=True, allow_infinity=True, width=64),
               st.integers(-(2 ** 70), 2 ** 70))


@SETTINGS
@given(st.lists(_f, max_size=64), st.sampled_from([", ", ",", " , ", ",\n"]))
def test_json_parser_matches_python(vals, sep):
    text = "[" + sep.join(json.dumps(v) for v in vals) + "]"
    got = torch.tensor(core().parse_json_f32(text.encode()), dtype=torch.float32)
    exp = torch.tensor([float(x) for x in json.loads(text)], dtype=torch.float64).to(torch.float32)
    assert core().json_array_len(text.encode()) == len(vals)
    assert torch.equal(torch.isnan(got), torch.isnan(exp))
    assert torch.equal(got.nan_to_num(), exp.nan_to_num())


@SETTINGS
@given(st.integers(1, 300), st.integers(1, 16), st.integers(1, 8))
def test_static_sharding_is_a_partition(n_parts, world, workers):
    owners = {}
    for r in range(world):
        for w in range(workers):
            for p in shard_partitions(n_parts, r, world, w, workers):
                assert p not in owners
                owners[p] = (r, w)
    assert sorted(owners) == list(range(n_parts))
    assert all(shard_owner(p, world, workers) == o for p, o in owners.items())
    # balance: ranks differ by at most one partition
    per_rank = [sum(1 for o in owners.values() if o[0] == r) for r in range(world)]
    assert max(per_rank) - min(per_rank) <= 1


@SETTINGS
@given(st.lists(st.integers(0, 40), min_size=1, max_size=20), st.integers(1, 48),
       st.sampled_from([torch.float32, torch.bfloat16, torch.int32]))
def test_reference_varlen_pads_and_truncates(lens, L, dtype):
    from torchkafka_amd.ops.collate import reference_varlen

    offs = torch.zeros(len(lens) + 1, dtype=torch.int32)
    offs[1:] = torch.tensor(lens).cumsum(0).to(torch.int32)
    vals = torch.arange(int(offs[-1]), dtype=torch.float32) + 1
    out, ln, mask = reference_varlen(offs, vals, dtype, L, pad_value=-7, return_mask=True)
    assert out.shape == (len(lens), L) and out.dtype == dtype
    for r, n in enumerate(lens):
        k = min(n, L)
        assert int(ln[r]) == k
        assert mask[r].sum() == k and bool(mask[r, :k].all())
        assert torch.equal(out[r, :k].float(), vals[int(offs[r]): int(offs[r]) + k].to(dtype).float())
        assert bool((out[r, k:].float() == -7).all())


@pytest.mark.parametrize("n", [0, 1, 5])
def test_json_len_consistent_with_parse(n):
    text = json.dumps([math.pi * i for i in range(n)]).encode()
    assert core().json_array_len(text) == len(core().parse_json_f32(text)) == n
