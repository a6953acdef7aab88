"""Ahead launches on their own native thread (Tuning.launch_thread, csrc/hip/torch_step.cpp
Launcher) on the GPU: the records, their decoded bits and the commits are the same as with the
launches made by the stepping thread, for fixed-width, JSON and var-len device decode, and a
corrupt RecordBatch is still never handed out.  The two runs of each case deliver the same
records; their decoded rows are compared bit for bit."""
import os

import pytest
import torch

from conftest import synth_f32

pytestmark = pytest.mark.gpu


def _dataset(schema):
    from torchkafka_amd import KafkaDataset

    class DS(KafkaDataset):
        pass

    DS.schema = schema
    return DS


def _bits(t: torch.Tensor) -> torch.Tensor:
    return t.view({1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[t.element_size()])


def _run(broker, topic, DS, bs, group, launch_thread, **kw):
    from torchkafka_amd import DeviceLoader, auto_commit

    dl = DeviceLoader(DS.placeholder(), bs, device="cuda:0", launch_thread=launch_thread,
                      worker_init_fn=DS.init_worker(topic, bootstrap_servers=broker.url, group_id=group,
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300), **kw)
    out = []
    for item in auto_commit(dl):
        out.append(tuple(t.clone() for t in item) if isinstance(item, tuple) else item.clone())
    torch.cuda.synchronize()
    return out, dl


def _rows(items):
    """Every delivered row's bytes (var-len rows cut to their length), sorted: the two runs may
    group records into batches differently, the records and their decoded bits must not differ."""
    out = []
    for item in items:
        if isinstance(item, tuple):
            x, lengths = item[0].cpu(), item[1].cpu()
            out += [bytes(_bits(x[i, :int(lengths[i])].contiguous()).numpy().tobytes()) for i in range(x.shape[0])]
        else:
            x = item.cpu()
            out += [bytes(_bits(x[i].contiguous()).numpy().tobytes()) for i in range(x.shape[0])]
    return sorted(out)


def _same(a, b):
    ra, rb = _rows(a), _rows(b)
    assert len(ra) == len(rb) and ra == rb


def test_launcher_fixed_width_same_batches_values_and_commits(broker):
    from torchkafka_amd import FixedWidth

    broker.create_topic("t", 4)
    broker.fill("t", 2000, "fixed_f32", size=64, records_per_batch=50)
    DS = _dataset(FixedWidth(torch.float32, (64,)))
    runs = {}
    for lt in (False, True):
        runs[lt], dl = _run(broker, "t", DS, 64, f"g{int(lt)}", lt, num_workers=1, in_order=True,
                            dtype=torch.float32)
        assert dl.plan.span
        assert broker.committed_offsets(f"g{int(lt)}", "t") == {p: 2000 for p in range(4)}
        assert dl.stats.batches == 125
        assert dl.stats.ahead_ns > 0  # groups were decoded ahead (by the launcher thread when lt)
    _same(runs[False], runs[True])
    x = torch.cat(runs[True]).cpu()
    seen = {(int(r[1]), int(r[0])) for r in x}
    assert len(seen) == 8000
    r = x[777]
    assert torch.equal(r, torch.tensor([synth_f32(int(r[1]), int(r[0]), j) for j in range(64)]))


def test_launcher_json_same_batches_and_commits(broker):
    from torchkafka_amd import JsonArray

    broker.create_topic("j", 2)
    broker.fill("j", 1500, "json_f32", size=16, max_size=256)
    DS = _dataset(JsonArray())
    runs = {}
    for lt in (False, True):
        runs[lt], dl = _run(broker, "j", DS, 256, f"g{int(lt)}", lt, num_workers=1, in_order=True,
                            dtype=torch.bfloat16)
        assert dl.plan.json_span and dl.plan.mirror  # the default JSON path: HBM mirror
        assert dl.stats.ahead_ns > 0
        assert broker.committed_offsets(f"g{int(lt)}", "j") == {0: 1500, 1: 1500}
    _same(runs[False], runs[True])


def test_launcher_varlen_tokens_same_batches(broker):
    from torchkafka_amd import VarLen

    broker.create_topic("v", 2)
    broker.fill("v", 1200, "tokens_i32", size=8, max_size=200)
    DS = _dataset(VarLen(torch.int32))
    runs = {}
    for lt in (False, True):
        runs[lt], dl = _run(broker, "v", DS, 128, f"g{int(lt)}", lt, num_workers=1, in_order=True,
                            dtype=torch.int64)
        assert dl.plan.var_span
        assert broker.committed_offsets(f"g{int(lt)}", "v") == {0: 1200, 1: 1200}
    _same(runs[False], runs[True])


def test_launcher_verify_deliver_never_yields_a_corrupt_batch(broker):
    from torchkafka_amd import DeviceLoader, FixedWidth, auto_commit
    from torchkafka_amd.client.errors import CorruptRecordException

    rpb, size, bad_rb = 16, 64, 9
    broker.create_topic("c", 1)
    broker.fill("c", 400, "fixed_f32", size=size, records_per_batch=rpb)
    pidx = broker.pidx("c", 0)
    log = broker.native.read_log(pidx, 0, broker.native.log_bytes(pidx))
    pos, k = 0, 0
    while k < bad_rb:
        pos += 12 + int.from_bytes(log[pos + 8:pos + 12], "big")
        k += 1
    path = os.path.join(broker.native.dir, f"p{pidx:05d}.log")
    with open(path, "r+b") as f:  # one flipped byte inside record values of RecordBatch bad_rb
        at = pos + 61 + 30 + size * 2
        f.seek(at)
        f.write(bytes([log[at] ^ 0x5A]))
    DS = _dataset(FixedWidth(torch.float32, (size,)))
    dl = DeviceLoader(DS.placeholder(), rpb, num_workers=1, device="cuda:0", launch_thread=True,
                      dtype=torch.float32,
                      worker_init_fn=DS.init_worker("c", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    seen = []
    with pytest.raises(CorruptRecordException, match="failed CRC check"):
        for x in auto_commit(dl):
            seen += x[:, 0].long().tolist()
    assert seen == list(range(bad_rb * rpb))
    assert broker.committed_offsets("g", "c").get(0) == bad_rb * rpb
