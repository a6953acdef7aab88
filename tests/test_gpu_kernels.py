"""Numerics of the gfx950 collate kernels against plain PyTorch references (bit-exact)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

FLOATS = [torch.float32, torch.bfloat16, torch.float16, torch.float8_e4m3fn]


def special_f32(n: int, seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g) * torch.exp2(torch.randint(-20, 20, (n,), generator=g).float())
    specials = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 1e-40, -1e-42, 448.0, 449.0,
                             464.0, 479.9, 480.0, 65504.0, 65520.0, 3.0e38, 2 ** -9, 2 ** -10, 0.0009765625,
                             1.0 + 2 ** -8, 1.0 + 3 * 2 ** -9, -3.5, 2 ** -6, 2 ** -7 * 1.5])
    k = min(n, specials.numel())
    x[:k] = specials[:k]
    return x


def bits(t: torch.Tensor) -> torch.Tensor:
    if t.element_size() == 1:
        return t.view(torch.uint8).to(torch.int32)
    if t.element_size() == 2:
        return t.view(torch.int16).to(torch.int32)
    return t.view(torch.int32)


def assert_same(out: torch.Tensor, ref: torch.Tensor):
    assert out.dtype == ref.dtype and out.shape == ref.shape
    o, r = out.cpu(), ref.cpu()
    if o.dtype.is_floating_point:
        on, rn = torch.isnan(o.float()), torch.isnan(r.float())
        assert torch.equal(on, rn), "NaN positions differ"
        keep = ~on
        assert torch.equal(bits(o)[keep], bits(r)[keep]), "values differ"
    else:
        assert torch.equal(o, r)


@pytest.mark.parametrize("dst", FLOATS)
@pytest.mark.parametrize("row", [256, 13, 8])
def test_fixed_cast_matches_torch(dst, row):
    from torchkafka_amd.ops.collate import collate_fixed

    rows = 37
    src = special_f32(rows * row, seed=row).view(rows, row)
    out = collate_fixed(src.cuda(), dst)
    torch.cuda.synchronize()
    assert_same(out, src.to(dst))


@pytest.mark.parametrize("dst", [torch.float32, torch.bfloat16, torch.float8_e4m3fn])
def test_fixed_normalize_fused(dst):
    from torchkafka_amd.ops.collate import collate_fixed, reference_fixed

    src = torch.randn(64, 256) * 3 + 1
    mean, std = torch.randn(256), torch.rand(256) + 0.5
    out = collate_fixed(src.cuda(), dst, normalize=(mean, std))
    ref = reference_fixed(src, dst, normalize=(mean, std))
    assert_same(out, ref)


@pytest.mark.parametrize("src_dt,dst", [(torch.bfloat16, torch.float32), (torch.float16, torch.bfloat16),
                                        (torch.uint8, torch.float32), (torch.uint8, torch.bfloat16),
                                        (torch.int32, torch.int64), (torch.int64, torch.int32),
                                        (torch.int8, torch.float16)])
def test_fixed_other_sources(src_dt, dst):
    from torchkafka_amd.ops.collate import collate_fixed

    if src_dt.is_floating_point:
        src = torch.randn(33, 64).to(src_dt)
    else:
        info = torch.iinfo(src_dt)
        src = torch.randint(max(info.min, -1000), min(info.max, 1000), (33, 64), dtype=torch.int64).to(src_dt)
    out = collate_fixed(src.cuda(), dst)
    assert_same(out, src.to(dst))


@pytest.mark.parametrize("rows", [1024, 1031])
def test_fixed_unrolled_tiles(rows):
    """>= 256*256*4 groups: the 4-deep unrolled kernel, including a ragged last tile."""
    from torchkafka_amd.ops.collate import collate_fixed

    src = special_f32(rows * 2048, seed=rows).view(rows, 2048)
    for dt in (torch.bfloat16, torch.float8_e4m3fn):
        assert_same(collate_fixed(src.cuda(), dt), src.to(dt))
    mean, std = torch.randn(2048), torch.rand(2048) + 0.5
    from torchkafka_amd.ops.collate import reference_fixed
    assert_same(collate_fixed(src.cuda(), torch.bfloat16, normalize=(mean, std)),
                reference_fixed(src, torch.bfloat16, normalize=(mean, std)))


def test_fixed_large_grid_stride():
    from torchkafka_amd.ops.collate import collate_fixed

    src = torch.randn(4096, 1024)  # 4M elements -> grid capped at 2048 blocks, grid-stride loop
    out = collate_fixed(src.cuda(), torch.bfloat16)
    assert_same(out, src.to(torch.bfloat16))


@pytest.mark.parametrize("dst", FLOATS + [torch.int32])
def test_varlen_pad_matches_reference(dst):
    from torchkafka_amd.ops.collate import collate_varlen, reference_varlen

    g = torch.Generator().manual_seed(3)
    lens = torch.randint(0, 300, (50,), generator=g)
    lens[0], lens[1], lens[2] = 0, 4097, 1  # empty row, a row spanning 3 chunks, single element
    offs = torch.zeros(51, dtype=torch.int32)
    offs[1:] = lens.cumsum(0).to(torch.int32)
    if dst == torch.int32:
        vals = torch.randint(-5000, 5000, (int(offs[-1]),), generator=g, dtype=torch.int32)
    else:
        vals = special_f32(int(offs[-1]), seed=5)
    L = int(lens.max())
    out, ln, mask = collate_varlen(offs.cuda(), vals.cuda(), dst, L=L, pad_value=-1, return_mask=True)
    r_out, r_ln, r_mask = reference_varlen(offs, vals, dst, L, pad_value=-1, return_mask=True)
    assert_same(out, r_out)
    assert torch.equal(ln.cpu(), r_ln)
    assert torch.equal(mask.cpu(), r_mask)


@pytest.mark.parametrize("src_dt,dst", [(torch.bfloat16, torch.float32), (torch.float16, torch.bfloat16),
                                        (torch.uint8, torch.int32), (torch.int64, torch.int32),
                                        (torch.int8, torch.float16)])
def test_varlen_narrow_and_wide_sources(src_dt, dst):
    """1/2-byte sources take the LDS-staged kernel (row starts not dword-aligned), 4/8-byte the direct one."""
    from torchkafka_amd.ops.collate import collate_varlen, reference_varlen

    g = torch.Generator().manual_seed(11)
    lens = torch.randint(0, 3000, (37,), generator=g)
    lens[0], lens[1] = 0, 2049
    offs = torch.zeros(38, dtype=torch.int32)
    offs[1:] = lens.cumsum(0).to(torch.int32)
    n = int(offs[-1])
    if src_dt.is_floating_point:
        vals = torch.randn(n, generator=g).to(src_dt)
    else:
        info = torch.iinfo(src_dt)
        vals = torch.randint(max(info.min, -100), min(info.max, 100), (n,), generator=g, dtype=torch.int64).to(src_dt)
    L = int(lens.max()) + 5
    out, ln, mask = collate_varlen(offs.cuda(), vals.cuda(), dst, L=L, pad_value=3, return_mask=True)
    r_out, r_ln, r_mask = reference_varlen(offs, vals, dst, L, pad_value=3, return_mask=True)
    assert_same(out, r_out)
    assert torch.equal(ln.cpu(), r_ln) and torch.equal(mask.cpu(), r_mask)


def test_varlen_truncating_width():
    from torchkafka_amd.ops.collate import collate_varlen, reference_varlen

    lens = torch.tensor([5, 17, 0, 9])
    offs = torch.zeros(5, dtype=torch.int32)
    offs[1:] = lens.cumsum(0).to(torch.int32)
    vals = torch.arange(int(offs[-1]), dtype=torch.float32)
    out, ln = collate_varlen(offs.cuda(), vals.cuda(), torch.bfloat16, L=8)
    r_out, r_ln = reference_varlen(offs, vals, torch.bfloat16, 8)
    assert_same(out, r_out)
    assert torch.equal(ln.cpu(), r_ln)


def test_extension_is_native():
    """The device path must be the compiled gfx950 extension, never a Python fallback."""
    from torchkafka_amd.ops import hip

    mod = hip()
    assert mod.__file__.endswith(".so")
    info = mod.device_info(0)
    assert "gfx950" in info["gcn_arch"], info


# ----------------------------------------------------------------------------- property-based (hypothesis)
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

_GPU_SETTINGS = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@_GPU_SETTINGS
@given(st.integers(0, 300), st.integers(1, 700), st.sampled_from(FLOATS), st.integers(0, 2 ** 16))
def test_fixed_property(rows, row, dst, seed):
    from torchkafka_amd.ops.collate import collate_fixed

    src = special_f32(max(rows * row, 1), seed=seed)[: rows * row].view(rows, row)
    out = collate_fixed(src.cuda(), dst)
    assert_same(out, src.to(dst))


@_GPU_SETTINGS
@given(st.lists(st.integers(0, 5000), min_size=1, max_size=64), st.sampled_from(FLOATS),
       st.one_of(st.none(), st.integers(1, 6000)), st.integers(0, 2 ** 16))
def test_varlen_property(lens, dst, L, seed):
    """Any length distribution (L=0 rows, one huge row, truncation) pads exactly like the torch reference."""
    from torchkafka_amd.ops.collate import collate_varlen, reference_varlen

    offs = torch.zeros(len(lens) + 1, dtype=torch.int32)
    offs[1:] = torch.tensor(lens).cumsum(0).to(torch.int32)
    vals = special_f32(max(int(offs[-1]), 1), seed=seed)[: int(offs[-1])]
    width = L if L is not None else max(max(lens), 1)
    out, ln, mask = collate_varlen(offs.cuda(), vals.cuda(), dst, L=width, pad_value=0.5, return_mask=True)
    r_out, r_ln, r_mask = reference_varlen(offs, vals, dst, width, pad_value=0.5, return_mask=True)
    assert_same(out, r_out)
    assert torch.equal(ln.cpu(), r_ln)
    assert torch.equal(mask.cpu(), r_mask)


_SERIAL_SCRIPT = r"""
import torch
from torchkafka_amd.ops.collate import collate_fixed, collate_varlen, reference_varlen
src = torch.randn(257, 333)
assert torch.equal(collate_fixed(src.cuda(), torch.bfloat16).cpu().view(torch.int16),
                   src.to(torch.bfloat16).view(torch.int16))
lens = torch.tensor([0, 4097, 1, 300, 2048])
offs = torch.zeros(6, dtype=torch.int32); offs[1:] = lens.cumsum(0).to(torch.int32)
vals = torch.randn(int(offs[-1]))
out, ln = collate_varlen(offs.cuda(), vals.cuda(), torch.float16, L=4097)
r, rl = reference_varlen(offs, vals, torch.float16, 4097)
assert torch.equal(out.cpu().view(torch.int16), r.view(torch.int16)) and torch.equal(ln.cpu(), rl)
print("OK")
"""


def test_kernels_under_serialized_launches():
    """re-run the kernels with launches serialised (AMD_SERIALIZE_KERNEL / HIP_LAUNCH_BLOCKING)
    so a missing stream dependency cannot hide behind asynchrony."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3", AMD_SERIALIZE_COPY="3", HIP_LAUNCH_BLOCKING="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _SERIAL_SCRIPT], env=env, cwd=root, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-2000:]
