"""The fixed-width decode kernel with each segment split over 2 or 4 workgroups
(TORCHKAFKA_SPAN_SPLIT / TORCHKAFKA_MIRROR_SPLIT, span_decode.hip step 0): the parts stage and
check disjoint byte ranges of a RecordBatch, and the last part to finish combines their CRCs.
The cases of tests/test_gpu_span.py that exercise the split's edges run again under each split:
values bit-exact with the host path (rows cut by part boundaries, 1- to 4-byte elements, RecordBatches
chained over segments, the HBM mirror), and a flipped byte caught in every part's range."""
import pytest
import torch

import test_gpu_span as base

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[2, 4])
def split(request, monkeypatch):
    monkeypatch.setenv("TORCHKAFKA_SPAN_SPLIT", str(request.param))
    monkeypatch.setenv("TORCHKAFKA_MIRROR_SPLIT", str(request.param))
    return request.param


@pytest.mark.parametrize("shape,src,dst,norm,bs,rpb,workers", [
    ((256,), torch.float32, torch.bfloat16, False, 64, 64, 2),
    ((13,), torch.float32, torch.float32, False, 33, 7, 2),
    ((40,), torch.bfloat16, torch.float32, False, 32, 5, 1),
    ((48,), torch.uint8, torch.float16, False, 32, 9, 1),
    ((64,), torch.float32, torch.bfloat16, True, 32, 16, 1),
    ((12000,), torch.float32, torch.bfloat16, False, 8, 4, 1),
    ((3,), torch.int32, torch.int64, False, 1000, 400, 1),
])
def test_split_decode_matches_host_path(broker, split, shape, src, dst, norm, bs, rpb, workers):
    base.test_device_decode_matches_host_path(broker, shape, src, dst, norm, bs, rpb, workers)


def test_split_is_in_effect(broker, split):
    from torchkafka_amd import DeviceLoader, FixedWidth, auto_commit

    broker.create_topic("t", 2)
    broker.fill("t", 256, "fixed_f32", size=256, records_per_batch=64)
    DS = base._dataset(FixedWidth(torch.float32, (256,)))
    dl = DeviceLoader(DS.placeholder(), 64, num_workers=1, device="cuda:0", decode="device",
                      worker_init_fn=DS.init_worker("t", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    it = iter(auto_commit(dl))
    x = next(it)
    assert dl._run.driver.span_split == split and dl._run.driver.mirror_split == split
    n = x.shape[0] + sum(y.shape[0] for y in it)
    assert n == 512


@pytest.mark.parametrize("size,rpb", [(64, 10), (12000, 4)])
def test_split_crc_failure_raises_before_commit(broker, split, size, rpb):
    base.test_device_decode_crc_failure_raises_before_commit(broker, size, rpb)


@pytest.mark.parametrize("frac", [0.02, 0.3, 0.55, 0.8, 0.99])
def test_split_catches_a_flip_in_every_part(broker, split, frac):
    """A 64-record RecordBatch of 1 KiB values (config 2's shape, ~66 KB: every part holds some of
    it); one byte flipped at `frac` of the way through its values."""
    from torchkafka_amd import DeviceLoader, FixedWidth, auto_commit
    from torchkafka_amd.client.errors import CorruptRecordException

    rpb, size, bad_rb = 64, 256, 3
    broker.create_topic("c", 1)
    broker.fill("c", rpb * 8, "fixed_f32", size=size, records_per_batch=rpb)
    pidx = broker.pidx("c", 0)
    log = broker.native.read_log(pidx, 0, broker.native.log_bytes(pidx))
    pos, k = 0, 0
    while k < bad_rb:
        pos += 12 + int.from_bytes(log[pos + 8:pos + 12], "big")
        k += 1
    rb_len = 12 + int.from_bytes(log[pos + 8:pos + 12], "big")
    base._corrupt(broker, pidx, pos + 61 + int((rb_len - 61) * frac))
    DS = base._dataset(FixedWidth(torch.float32, (size,)))
    dl = DeviceLoader(DS.placeholder(), rpb, num_workers=1, device="cuda:0", decode="device", coalesce=4,
                      worker_init_fn=DS.init_worker("c", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    seen = 0
    with pytest.raises(CorruptRecordException, match=f"offset {bad_rb * rpb} .*failed CRC check"):
        for x in auto_commit(dl):
            seen += x.shape[0]
    assert seen == bad_rb * rpb
    assert broker.committed_offsets("g", "c").get(0) == bad_rb * rpb


@pytest.mark.parametrize("chunk_mib,chunks,rpb,size", [(1, 2, 16, 256), (1, 3, 4, 12000)])
def test_split_decode_through_hbm_mirror(broker, split, chunk_mib, chunks, rpb, size):
    base.test_device_decode_through_hbm_mirror(broker, chunk_mib, chunks, rpb, size)
