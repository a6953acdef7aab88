"""Decode segments split over P workgroups ("parts": span_device.h ``Part`` / ``crc_finish``).

A launch whose segments are all read from the HBM mirror gives each segment P workgroups, each
streaming windows [q*nw/P, (q+1)*nw/P) of it; each part shifts its CRC32C to the segment's end and
XORs it into an accumulator set of the launch, and the last part to arrive gives the verdict
(TORCHKAFKA_SPAN_PARTS, default 8).  Segments are split only under a mirror whose launches wait
for copies in flight -- fixed-width decode's; JSON / var-len keep the no-wait mirror and one
workgroup per segment (driver.h mirror_splits, profiles/r06_s21, r06_s23).  Run
under P = 1, 2, 4 and 8: values bit-exact with the host path through the mirror (rows cut by part
boundaries, parts with no window, RecordBatches chained over segments), a flipped byte caught in
every part's range with the batches before it committed, and the split actually in effect.
The CPU side of the combination is tests/test_span_decode.py (crc32c_span_emulate)."""
import pytest
import torch

import test_gpu_span as base

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[1, 2, 4, 8])
def parts(request, monkeypatch):
    monkeypatch.setenv("TORCHKAFKA_SPAN_PARTS", str(request.param))
    return request.param


def _loader(broker, topic, DS, bs, group, **kw):
    from torchkafka_amd import DeviceLoader

    return DeviceLoader(DS.placeholder(), bs, device="cuda:0", decode="device", h2d="dma",
                        worker_init_fn=DS.init_worker(topic, bootstrap_servers=broker.url, group_id=group,
                                                      auto_offset_reset="earliest", consumer_timeout_ms=300), **kw)


@pytest.mark.parametrize("shape,src,dst,bs,rpb", [
    ((256,), torch.float32, torch.bfloat16, 64, 64),    # config 2's rows, 66 KB RecordBatches
    ((13,), torch.float32, torch.float32, 33, 7),       # 52-byte rows: rows cut by window boundaries
    ((48,), torch.uint8, torch.float16, 32, 9),         # 1-byte elements
    ((12000,), torch.float32, torch.bfloat16, 8, 4),    # 192 KB RecordBatches chained over segments
    ((3,), torch.int32, torch.int64, 1000, 400),        # one short segment: parts without a window
])
def test_parts_decode_through_mirror_matches_host_path(broker, parts, shape, src, dst, bs, rpb):
    from torchkafka_amd import FixedWidth, auto_commit

    numel = 1
    for d in shape:
        numel *= d
    esize = torch.empty((), dtype=src).element_size()
    n = 120 if numel < 1000 else 24
    broker.create_topic("t", 3)
    base._produce_random(broker, "t", 3, n, numel * esize, rpb=rpb)
    DS = base._dataset(FixedWidth(src, shape))
    a, _ = base._run(broker, "t", DS, "host", bs, "gh", num_workers=2, dtype=dst, in_order=True, coalesce=4)
    dl = _loader(broker, "t", DS, bs, "gm", num_workers=2, dtype=dst, in_order=True, coalesce=4)
    assert dl.plan.mirror
    b = torch.cat([x.clone() for x in auto_commit(dl)])
    torch.cuda.synchronize()
    assert a.shape == b.shape == (3 * n, *shape)
    assert torch.equal(base._bits(a), base._bits(b))
    assert broker.committed_offsets("gm", "t") == {0: n, 1: n, 2: n}
    st = dl.stats_summary()
    assert st["mirror_copies"] > 0
    # fixed-width decode: the mirror waits for its copies, so a launch reads HBM and is split unless
    # one of its buffers was busy
    assert st["mirror_pending_fallbacks"] == 0, st
    if parts == 1:
        assert st["split_launches"] == 0
    else:
        assert st["split_launches"] > 0 or st["mirror_fallbacks"] > 0, st  # (a busy buffer: whole)


@pytest.mark.parametrize("frac", [0.02, 0.3, 0.55, 0.8, 0.99])
def test_parts_catch_a_flip_in_every_part(broker, parts, frac):
    """64-record RecordBatches of 1 KiB values (~66 KB, so each spans segments whose windows are
    split over the parts); one byte of RecordBatch 3 flipped at ``frac`` of its values."""
    from torchkafka_amd import FixedWidth, auto_commit
    from torchkafka_amd.client.errors import CorruptRecordException

    rpb, size, bad_rb = 64, 256, 3
    broker.create_topic("c", 1)
    broker.fill("c", rpb * 8, "fixed_f32", size=size, records_per_batch=rpb)
    pidx = broker.pidx("c", 0)
    log = broker.native.read_log(pidx, 0, broker.native.log_bytes(pidx))
    pos = 0
    for _ in range(bad_rb):
        pos += 12 + int.from_bytes(log[pos + 8:pos + 12], "big")
    rb_len = 12 + int.from_bytes(log[pos + 8:pos + 12], "big")
    base._corrupt(broker, pidx, pos + 61 + int((rb_len - 61) * frac))
    DS = base._dataset(FixedWidth(torch.float32, (size,)))
    dl = _loader(broker, "c", DS, rpb, "g", num_workers=1, coalesce=4)
    seen = 0
    with pytest.raises(CorruptRecordException, match=f"offset {bad_rb * rpb} .*failed CRC check"):
        for x in auto_commit(dl):
            seen += x.shape[0]
    assert seen == bad_rb * rpb
    assert broker.committed_offsets("g", "c").get(0) == bad_rb * rpb


def test_parts_var_len_through_mirror(broker, parts):
    """VarLen token rows decoded from the HBM mirror (h2d='dma') under each split."""
    base.test_var_span_matches_host_path(broker, torch.int32, torch.int64, (0, 300), 0, 0, {"h2d": "dma"})
