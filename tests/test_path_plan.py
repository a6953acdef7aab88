"""PathPlan (loader/path_plan.py): the data path a DeviceLoader takes, decided once from its
configuration.  A pure function of the configuration, so the whole decision table is checked here
on the CPU -- the GPU tests then exercise each path's kernels.

The reference has one path (kafka-python iterator -> _process -> DataLoader collate,
/root/reference/src/kafka_dataset.py:147-171); these are the device paths SURVEY §2.6 adds."""
import pytest
import torch

from torchkafka_amd import FixedWidth, JsonArray, VarLen
from torchkafka_amd.loader.path_plan import PathPlan, ZERO_COPY_MAX_BYTES


def plan(schema=None, device="cuda", native=True, decode="auto", h2d="auto", json_parse="auto", synthetic=True,
         overridden=False, return_info=False, drop_last=False, json_count="auto"):
    return PathPlan.build(device_type=device, schema=schema, native=native, decode=decode, h2d=h2d,
                          json_parse=json_parse, synthetic_commits=synthetic, process_overridden=overridden,
                          return_info=return_info, drop_last=drop_last, json_count_mode=json_count)


FIXED, VAR, JSON = FixedWidth(torch.float32, (16,)), VarLen(torch.int32, max_len=64), JsonArray()


@pytest.mark.parametrize("schema,want", [(FIXED, "span"), (VAR, "var_span"), (JSON, "json_span")])
def test_auto_decodes_on_the_device_from_the_logs(schema, want):
    p = plan(schema)
    assert getattr(p, want) and p.device_decode
    assert p.mirror == (schema is JSON)  # JSON rows through the HBM mirror
    assert p.resolve_h2d(1 << 30) == "zerocopy"  # row tables are read once, in place


@pytest.mark.parametrize("kw", [dict(device="cpu"), dict(native=False), dict(synthetic=False),
                                dict(overridden=True), dict(decode="host")])
def test_device_decode_needs_gpu_native_synthetic_and_the_schema(kw):
    p = plan(FIXED, **kw)
    assert not p.device_decode


def test_mirror_default_for_json_only():
    """'auto' takes the HBM mirror for JSON rows (46-52 M rec/s against 38 M zero-copy, and under
    the RCCL lockstep 46-52 M against 33 M) and stays zero-copy for fixed-width and var-len rows
    (var-len: 45-47 M zero-copy against 42-43 M mirrored, 42-47 M against 31-37 M under the
    lockstep; profiles/r05_s35_mirror_rccl); 'dma' always mirrors, 'zerocopy' never."""
    for schema in (FIXED, VAR, JSON):
        assert plan(schema, h2d="dma").mirror
        assert not plan(schema, h2d="zerocopy").mirror
    assert not plan(FIXED, h2d="auto").mirror
    assert not plan(VAR, h2d="auto").mirror and plan(JSON, h2d="auto").mirror
    assert not plan(FIXED, h2d="dma", decode="host").mirror  # nothing read from the logs
    assert not plan(JSON, decode="host").mirror and not plan(VAR, device="cpu").mirror


def test_generic_paths_pick_h2d_by_slot_size():
    p = plan(FIXED, decode="host")
    assert p.fast_path and not p.device_decode
    assert p.resolve_h2d(ZERO_COPY_MAX_BYTES) == "zerocopy" and p.resolve_h2d(ZERO_COPY_MAX_BYTES + 1) == "dma"
    assert plan(FIXED, return_info=True).fast_path is False
    assert plan(VAR, drop_last=True).varlen_fast is False


def test_json_parse_and_count_choices():
    assert plan(JSON, json_parse="host").json_device is False
    assert plan(JsonArray(skip_bad=True)).json_device is False  # dropping a row needs the host parser
    assert plan(JSON).json_count and not plan(JSON, json_count="host").json_count
    assert not plan(JsonArray(min_len=2)).json_count  # a filter needs the workers' counts
    assert plan(JSON, decode="host").json_device and not plan(JSON, decode="host").json_span


@pytest.mark.parametrize("kw,msg", [
    (dict(schema=FIXED, decode="device", device="cpu"), "decode='device' needs a CUDA device"),
    (dict(schema=VAR, decode="device", synthetic=False), "decode='device' for VarLen"),
    (dict(schema=JSON, decode="device", synthetic=False), "synthetic broker"),
    (dict(schema=JsonArray(skip_bad=True), json_parse="device"), "skip_bad=False"),
    (dict(schema=JsonArray(min_len=3), json_count="device"), "cannot drop rows"),
    (dict(schema=FIXED, h2d="direct", return_info=True), "h2d='direct' needs a CUDA device"),
    (dict(schema=FIXED, h2d="direct", synthetic=False), "h2d='direct' needs the synthetic broker"),
])
def test_invalid_combinations_raise_at_construction(kw, msg):
    with pytest.raises(ValueError, match=msg):
        plan(**kw)


def test_direct_gather_and_ring_sizing():
    p = plan(FIXED, h2d="direct")
    assert p.direct and not p.span and p.resolve_h2d(10) == "direct"
    assert plan(FIXED).slots_per_worker(4096, 4) == 16            # row tables: deep ring
    assert plan(FIXED).slots_per_worker(4096, 4, deep=True) == 64  # under an RCCL lockstep: deeper
    assert plan(FIXED, decode="host").slots_per_worker(1 << 20, 4) == 8
    assert plan(FIXED, decode="host").slots_per_worker(64 << 20, 4) == 4
    assert plan(FIXED, decode="host").layout_capacity(256, FIXED) == 256 * 64
    assert plan(FIXED).describe()["decode"] == "device from the pinned logs"
