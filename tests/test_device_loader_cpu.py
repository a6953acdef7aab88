"""DeviceLoader semantics on the CPU device: ring, workers, exact commits, sharding, errors."""
import os

import pytest
import torch

from conftest import synth_f32
from torchkafka_amd import DeviceLoader, FixedWidth, JsonArray, KafkaDataset, VarLen, auto_commit
from torchkafka_amd.loader import WorkerError


class Vec16(KafkaDataset):
    schema = FixedWidth(torch.float32, (16,))


class Vec16Lenient(KafkaDataset):
    schema = FixedWidth(torch.float32, (16,), skip_bad=True)


class Json(KafkaDataset):
    schema = JsonArray(min_len=3)


class Tokens(KafkaDataset):
    schema = VarLen(torch.int32, max_len=20)


class Doubled(KafkaDataset):
    def _process(self, record):
        t = torch.frombuffer(bytearray(record.value), dtype=torch.float32)
        return None if int(t[0]) % 4 == 0 else t * 2


class Ragged(KafkaDataset):
    def _process(self, record):
        n = int(record.offset % 5)
        return torch.arange(n, dtype=torch.int64) + record.offset


class Crashy(KafkaDataset):
    def _process(self, record):
        if record.offset == 5:
            os._exit(3)
        return torch.zeros(2)


def init(ds_cls, broker, topic="t", group="g", **kw):
    d = dict(bootstrap_servers=broker.url, group_id=group, auto_offset_reset="earliest", consumer_timeout_ms=250)
    d.update(kw)
    return ds_cls.init_worker(topic, **d)


def loader(ds_cls, broker, bs, workers=2, topic="t", group="g", consumer_kw=None, **kw):
    return DeviceLoader(ds_cls.placeholder(), bs, num_workers=workers, device="cpu",
                        worker_init_fn=init(ds_cls, broker, topic, group, **(consumer_kw or {})), **kw)


def check_rows(x):
    for row in x:
        o, p = int(row[0]), int(row[1])
        assert row.tolist() == [synth_f32(p, o, j) for j in range(x.shape[1])]


@pytest.mark.parametrize("workers", [1, 2, 4])
def test_fixed_width_all_records_once(broker, workers):
    broker.create_topic("t", 4)
    broker.fill("t", 250, "fixed_f32", size=16, records_per_batch=32)
    seen = set()
    for x in auto_commit(loader(Vec16, broker, 64, workers)):
        assert x.dtype == torch.float32 and x.shape[1] == 16
        check_rows(x)
        for o, p in x[:, :2].long().tolist():
            assert (p, o) not in seen
            seen.add((p, o))
    assert len(seen) == 1000
    assert broker.committed_offsets("g", "t") == {p: 250 for p in range(4)}


def test_exact_commit_of_each_finished_batch(broker):
    broker.create_topic("t", 2)
    broker.fill("t", 100, "fixed_f32", size=16)
    dl = loader(Vec16, broker, 20, workers=2, return_info=True, slots_per_worker=4)
    gen = auto_commit(dl)
    b1 = next(gen)
    assert broker.committed_offsets("g", "t") == {0: None, 1: None}  # nothing finished yet
    next(gen)
    expect = {pidx: nxt for pidx, _f, nxt, _c in b1.watermarks}
    got = {broker.pidx("t", p): o for p, o in broker.committed_offsets("g", "t").items() if o is not None}
    assert got == expect  # exactly batch 1, despite the workers having prefetched further
    gen.close()  # like a `break`: the second batch is not committed
    assert {broker.pidx("t", p): o for p, o in broker.committed_offsets("g", "t").items() if o is not None} == expect


def test_manual_mode_and_commit(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 50, "fixed_f32", size=16)
    dl = loader(Vec16, broker, 10, workers=1)
    it = iter(dl)
    next(it), next(it)
    assert broker.committed("g", "t", 0) is None  # plain iteration never commits
    dl.commit()
    assert broker.committed("g", "t", 0) == 20
    it.close()


def test_resume_from_committed_offsets(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 60, "fixed_f32", size=16)
    gen = auto_commit(loader(Vec16, broker, 10, workers=1))
    first = [next(gen) for _ in range(3)]
    gen.close()  # batches 1 and 2 committed, batch 3 not
    assert broker.committed("g", "t", 0) == 20
    rest = torch.cat(list(auto_commit(loader(Vec16, broker, 10, workers=1))))
    assert rest[:, 0].long().tolist() == list(range(20, 60))  # batch 3 is re-delivered (at-least-once)
    assert torch.equal(first[2], rest[:10])


def test_drop_last_and_in_order(broker):
    broker.create_topic("t", 2)
    broker.fill("t", 35, "fixed_f32", size=16)
    xs = list(auto_commit(loader(Vec16, broker, 10, workers=2, drop_last=True, in_order=True)))
    assert all(x.shape[0] == 10 for x in xs) and len(xs) == 6
    assert broker.committed_offsets("g", "t") == {0: 35, 1: 35}  # dropped records still consumed


def test_bad_record_raises_in_main(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 5, "fixed_f32", size=16)
    broker.produce("t", [b"short"])
    with pytest.raises(WorkerError, match="does not match the fixed-width schema"):
        list(loader(Vec16, broker, 4, workers=1))


def test_skip_bad_and_nulls_are_skipped_but_committed(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 5, "fixed_f32", size=16)
    broker.produce("t", [b"short", None])
    broker.fill("t", 3, "fixed_f32", size=16)
    xs = torch.cat(list(auto_commit(loader(Vec16Lenient, broker, 4, workers=1))))
    assert xs[:, 0].long().tolist() == [0, 1, 2, 3, 4, 7, 8, 9]
    assert broker.committed("g", "t", 0) == 10


def test_json_min_len_filter(broker):
    from torchkafka_amd.client import KafkaConsumer

    broker.create_topic("t", 2)
    broker.fill("t", 80, "json_f32", size=0, max_size=9)
    rows = {}
    for x, lens in auto_commit(loader(Json, broker, 16, workers=2, dtype=torch.float32)):
        assert x.shape[1] % 8 == 0  # pad_multiple
        for i in range(x.shape[0]):
            n = int(lens[i])
            assert n >= 3
            assert bool((x[i, n:] == 0).all())
            rows.setdefault(n, []).append(tuple(x[i, :n].tolist()))
    ref = {}
    c = KafkaConsumer("t", bootstrap_servers=broker.url, auto_offset_reset="earliest", consumer_timeout_ms=100)
    for r in c:
        t = Json.schema.process(r)
        if t is not None:
            ref.setdefault(t.numel(), []).append(tuple(t.tolist()))
    assert {k: sorted(v) for k, v in rows.items()} == {k: sorted(v) for k, v in ref.items()}
    assert broker.committed_offsets("g", "t") == {0: 80, 1: 80}


def test_varlen_tokens_truncate_and_pad(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 40, "tokens_i32", size=1, max_size=40)
    n = 0
    for x, lens, mask in loader(Tokens, broker, 8, workers=1, dtype=torch.int64, pad_value=-1, return_mask=True):
        assert x.dtype == torch.int64 and int(lens.max()) <= 20
        assert torch.equal(mask, torch.arange(x.shape[1])[None, :] < lens[:, None])
        assert bool((x[~mask] == -1).all())
        n += x.shape[0]
    assert n == 40


def test_generic_process_path_dense_and_ragged(broker):
    broker.create_topic("t", 2)
    broker.fill("t", 40, "fixed_f32", size=8)
    xs = torch.cat(list(auto_commit(loader(Doubled, broker, 6, workers=2))))
    assert xs.shape == (60, 8)
    assert bool(((xs[:, 0] / 2) % 4 != 0).all())
    assert broker.committed_offsets("g", "t") == {0: 40, 1: 40}
    total = 0
    for x, lens in auto_commit(loader(Ragged, broker, 7, workers=1, group="g2")):
        for i in range(x.shape[0]):
            n = int(lens[i])
            off = int(x[i, 0]) if n else None
            if n:
                assert x[i, :n].tolist() == list(range(off, off + n))
        total += x.shape[0]
    assert total == 80


def test_worker_death_is_detected(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 20, "fixed_f32", size=2)
    with pytest.raises(WorkerError, match="exited unexpectedly"):
        list(loader(Crashy, broker, 4, workers=1))


def test_more_workers_than_partitions(broker):
    broker.create_topic("t", 2)
    broker.fill("t", 30, "fixed_f32", size=16)
    xs = torch.cat(list(auto_commit(loader(Vec16, broker, 8, workers=5))))
    assert xs.shape[0] == 60


def test_static_sharding_across_ranks(broker):
    broker.create_topic("t", 8)
    broker.fill("t", 20, "fixed_f32", size=16)
    owned = {}
    for rank in range(2):
        dl = loader(Vec16, broker, 16, workers=2, rank=rank, world_size=2, lockstep=False)
        parts = set()
        for x in auto_commit(dl):
            parts |= set(x[:, 1].long().tolist())
        owned[rank] = parts
    assert owned[0] == {0, 2, 4, 6} and owned[1] == {1, 3, 5, 7}
    assert broker.committed_offsets("g", "t") == {p: 20 for p in range(8)}


def test_group_sharding_mode(broker):
    broker.create_topic("t", 4)
    broker.fill("t", 25, "fixed_f32", size=16)
    xs = torch.cat(list(loader(Vec16, broker, 10, workers=2, sharding="group",
                               consumer_kw={"consumer_timeout_ms": 600})))
    assert sorted(map(tuple, xs[:, :2].long().tolist())) == sorted((o, p) for p in range(4) for o in range(25))


def test_normalize_and_bf16_on_cpu(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 16, "fixed_f32", size=16)
    mean, std = torch.arange(16.0), torch.full((16,), 2.0)
    x = torch.cat(list(loader(Vec16, broker, 16, workers=1, normalize=(mean, std))))
    raw = torch.tensor([[synth_f32(0, o, j) for j in range(16)] for o in range(16)])
    assert torch.allclose(x, (raw - mean) / std)
    xb = torch.cat(list(loader(Vec16, broker, 16, workers=1, dtype=torch.bfloat16, group="g3")))
    assert xb.dtype == torch.bfloat16 and torch.equal(xb, raw.to(torch.bfloat16))


def test_stats_and_commit_latency(broker):
    broker.create_topic("t", 2)
    broker.fill("t", 64, "fixed_f32", size=16)
    dl = loader(Vec16, broker, 16, workers=2)
    list(auto_commit(dl))
    s = dl.stats.summary()
    assert s["records"] == 128 and s["batches"] == 8 and s["commits"] >= 8
    assert s["commit_p99_us"] > 0


def test_len_is_undefined(broker):
    with pytest.raises(TypeError):
        len(DeviceLoader(Vec16.placeholder(), 4, num_workers=1, device="cpu"))


def test_state_dict_round_trip_resumes_exactly(broker):
    """Checkpoint = committed offsets; load_state_dict rewinds the group to them."""
    import json

    broker.create_topic("t", 2)
    broker.fill("t", 200, "fixed_f32", size=16, records_per_batch=10)
    dl = loader(Vec16, broker, 20, workers=1)
    it = iter(auto_commit(dl))
    seen = []
    for _ in range(5):
        seen.append(next(it))
    next(it)  # finishes (and commits) the 5th batch
    it.close()
    state = json.loads(json.dumps(dl.state_dict()))  # survives a JSON checkpoint
    assert state["group_id"] == "g"
    snap = {int(p): o for p, o in state["offsets"]["t"].items()}
    assert sum(snap.values()) >= 100
    # keep consuming: the group moves past the checkpoint
    for _ in auto_commit(loader(Vec16, broker, 20, workers=1)):
        pass
    assert broker.committed_offsets("g", "t") == {0: 200, 1: 200}
    # resume from the checkpoint: the first records delivered are exactly the checkpoint's positions
    dl2 = loader(Vec16, broker, 20, workers=1)
    dl2.load_state_dict(state)
    assert broker.committed_offsets("g", "t") == snap
    firsts = {}
    for x in auto_commit(dl2):
        for o, p in x[:, :2].long().tolist():
            firsts.setdefault(p, o)
    assert firsts == {p: o for p, o in snap.items() if o < 200}
    with pytest.raises(ValueError):
        dl2.load_state_dict({"version": 99, "offsets": {}})


def _direct(ds_cls, broker, topic="t", group="g", **kw):
    """The reference's single-process construction: the dataset owns its consumer."""
    d = dict(bootstrap_servers=broker.url, group_id=group, auto_offset_reset="earliest", consumer_timeout_ms=250)
    d.update(kw)
    return ds_cls(topic, **d)


def test_single_process_mode_exact_commits(broker):
    """num_workers=0 (reference auto_commit.py:49-58): no worker processes; a thread of this process
    packs the ring with the dataset's own consumer; every batch is committed once finished."""
    import multiprocessing as mp

    broker.create_topic("t", 3)
    broker.fill("t", 50, "fixed_f32", size=16, records_per_batch=20)
    dl = DeviceLoader(_direct(Vec16, broker), 16, num_workers=0, device="cpu")
    children = len(mp.active_children())
    seen = set()
    gen = auto_commit(dl)
    first = next(gen)
    assert len(mp.active_children()) == children  # nothing was forked
    for x in [first, *gen]:
        check_rows(x)
        seen |= {tuple(r) for r in x[:, :2].long().tolist()}
    assert len(seen) == 150
    assert broker.committed_offsets("g", "t") == {0: 50, 1: 50, 2: 50}


def test_single_process_mode_break_and_resume(broker):
    broker.create_topic("t", 1)
    broker.fill("t", 60, "fixed_f32", size=16)
    ds = _direct(Vec16, broker)
    for i, _x in enumerate(auto_commit(DeviceLoader(ds, 10, num_workers=0, device="cpu"))):
        if i == 2:
            break
    assert broker.committed("g", "t", 0) == 20  # batches 0 and 1 finished; the break skips batch 2
    ds.close()
    rest = torch.cat(list(auto_commit(DeviceLoader(_direct(Vec16, broker), 10, num_workers=0, device="cpu"))))
    assert sorted(rest[:, 0].long().tolist()) == list(range(20, 60))
    assert broker.committed("g", "t", 0) == 60


def test_single_process_mode_generic_process(broker):
    broker.create_topic("t", 2)
    broker.fill("t", 40, "fixed_f32", size=16)
    xs = torch.cat(list(auto_commit(DeviceLoader(_direct(Doubled, broker), 7, num_workers=0, device="cpu"))))
    offs = sorted((xs[:, 0] / 2).long().tolist())
    assert len(offs) == 60 and all(o % 4 for o in offs)
    assert broker.committed_offsets("g", "t") == {0: 40, 1: 40}


def test_single_process_mode_argument_errors(broker):
    broker.create_topic("t", 1)
    with pytest.raises(ValueError, match=r"num_workers=0\) needs a dataset with its consumer"):
        DeviceLoader(Vec16.placeholder(), 8, num_workers=0, device="cpu")
    with pytest.raises(ValueError, match="worker_init_fn is not used"):
        DeviceLoader(_direct(Vec16, broker), 8, num_workers=0, device="cpu", worker_init_fn=init(Vec16, broker))
    with pytest.raises(ValueError, match="num_workers must be >= 0"):
        DeviceLoader(Vec16.placeholder(), 8, num_workers=-1, device="cpu")


def test_commit_latency_is_measured_per_batch(broker):
    """commit latency = the user's request of batch k+1 -> batch k's offsets stored."""
    broker.create_topic("t", 2)
    broker.fill("t", 100, "fixed_f32", size=16)
    dl = loader(Vec16, broker, 20, workers=2)
    n = sum(1 for _ in auto_commit(dl))
    s = dl.stats_summary()
    assert n == 10 and s["commit_latency_samples"] == n
    assert 0 < s["commit_latency_p50_us"] <= s["commit_latency_p99_us"] <= s["commit_latency_max_us"]


# ---- structured samples: (features, label), dicts, lists -- as default_collate builds them

class Pair(KafkaDataset):
    """The reference README's shape: a feature tensor and a label."""

    def _process(self, record):
        v = torch.frombuffer(bytearray(record.value), dtype=torch.float32)
        return v[2:8].clone(), int(v[0]) % 3  # (features, python int label)


class Nested(KafkaDataset):
    def _process(self, record):
        v = torch.frombuffer(bytearray(record.value), dtype=torch.float32)
        if int(v[0]) % 5 == 4:
            return None  # skipped, still committed (B6)
        return {"x": v[2:6].view(2, 2).clone(), "meta": [torch.tensor([record.partition, record.offset]),
                                                        float(v[2])],
                "key": f"p{record.partition}o{record.offset}", "ok": True}


def _reference_batches(ds_cls, broker, bs, group):
    """What the reference's DataLoader + default_collate deliver for the same records."""
    from torch.utils.data import DataLoader

    ds = ds_cls("t", bootstrap_servers=broker.url, group_id=group, auto_offset_reset="earliest",
                consumer_timeout_ms=250)
    return list(DataLoader(ds, batch_size=bs))


@pytest.mark.parametrize("workers", [0, 1])
def test_structured_samples_match_default_collate(broker, workers):
    broker.create_topic("t", 1)
    broker.fill("t", 50, "fixed_f32", size=8)
    for cls in (Pair, Nested):
        ref = _reference_batches(cls, broker, 8, f"ref-{cls.__name__}")
        if workers:
            dl = loader(cls, broker, 8, workers=1, group=f"dl-{cls.__name__}")
        else:
            dl = DeviceLoader(cls("t", bootstrap_servers=broker.url, group_id=f"dl-{cls.__name__}",
                                  auto_offset_reset="earliest", consumer_timeout_ms=250), 8, num_workers=0,
                              device="cpu")
        got = list(auto_commit(dl))
        assert len(got) == len(ref)
        for a, b in zip(got, ref):
            fa, fb = torch.utils._pytree.tree_flatten(a), torch.utils._pytree.tree_flatten(b)
            assert fa[1] == fb[1]  # same structure (tuple / dict / list nesting, keys)
            for x, y in zip(fa[0], fb[0]):
                if isinstance(y, torch.Tensor):
                    assert x.dtype == y.dtype and torch.equal(x, y)
                else:
                    assert x == y
        committed = broker.committed_offsets(f"dl-{cls.__name__}", "t")
        assert committed == {0: 50}


def test_structured_samples_errors(broker):
    class Mixed(KafkaDataset):
        def _process(self, record):
            return (torch.zeros(2),) if record.offset % 2 else (torch.zeros(2), 1)

    class Ragged2(KafkaDataset):
        def _process(self, record):
            return {"x": torch.zeros(1 + record.offset % 2)}

    broker.create_topic("t", 1)
    broker.fill("t", 10, "fixed_f32", size=8)
    with pytest.raises(WorkerError, match="share their structure"):
        list(auto_commit(loader(Mixed, broker, 4, workers=1)))
    with pytest.raises(WorkerError, match="equal size"):
        list(auto_commit(loader(Ragged2, broker, 4, workers=1, group="g2")))


# ---- record fields beside the value: FixedWidth(...) + Key() + Timestamp()

def _produce_keyed(broker, n=60, parts=2, key_kind="be"):
    import struct

    from torchkafka_amd import KafkaProducer

    prod = KafkaProducer(bootstrap_servers=broker.url, linger_ms=0, batch_size=4096)
    for i in range(n):
        p = i % parts
        v = torch.arange(8, dtype=torch.float32) + i
        key = (struct.pack(">q", 1000 + i) if key_kind == "be" else str(1000 + i).encode()) if i % 7 else None
        prod.send("t", value=v.numpy().tobytes(), key=key, partition=p, timestamp_ms=1_700_000_000_000 + i)
    prod.flush()


@pytest.mark.parametrize("workers", [0, 2])
def test_key_and_timestamp_fields_ride_with_the_values(broker, workers):
    from torchkafka_amd import Key, Timestamp

    class Labelled(KafkaDataset):
        schema = FixedWidth(torch.float32, (8,)) + Timestamp() + Key("be", default=-7)

    broker.create_topic("t", 2)
    _produce_keyed(broker)
    kw = dict(bootstrap_servers=broker.url, group_id="g", auto_offset_reset="earliest", consumer_timeout_ms=250)
    if workers:
        dl = DeviceLoader(Labelled.placeholder(), 8, num_workers=workers, device="cpu",
                          worker_init_fn=Labelled.init_worker("t", **kw))
    else:
        dl = DeviceLoader(Labelled("t", **kw), 8, num_workers=0, device="cpu")
    seen = 0
    for x, ts, key in auto_commit(dl):
        assert ts.dtype == key.dtype == torch.int64 and ts.shape == key.shape == (x.shape[0],)
        for row, t, k in zip(x, ts.tolist(), key.tolist()):
            i = int(row[0])
            assert t == 1_700_000_000_000 + i
            assert k == (1000 + i if i % 7 else -7)
        seen += x.shape[0]
    assert seen == 60 and broker.committed_offsets("g", "t") == {0: 30, 1: 30}
    # the per-record path (torch DataLoader compat) gives the same fields
    rec = Labelled.schema.process(type("R", (), {"value": torch.zeros(8).numpy().tobytes(), "key": b"\0" * 8,
                                                   "timestamp": 5, "offset": 0})())
    assert rec[1].item() == 5 and rec[2].item() == 0


def test_ascii_keys_and_schema_validation():
    from torchkafka_amd import Key, Timestamp, VarLen
    from torchkafka_amd.ops.native import core

    assert core().key_int64(b"-42", 2, -1) == -42 and core().key_int64(b"4x", 2, -1) == -1
    assert core().key_int64(None, 0, 9) == 9 and core().key_int64(b"\0" * 7 + b"\x05", 0, -1) == 5
    # 19-digit keys: the int64 range is exact at both ends, one past it is the default (no overflow)
    k = core().key_int64
    assert k(b"9223372036854775807", 2, -1) == 2**63 - 1
    assert k(b"-9223372036854775808", 2, -1) == -2**63
    assert k(b"9223372036854775808", 2, -1) == -1 and k(b"-9223372036854775809", 2, -1) == -1
    assert k(b"9999999999999999999", 2, 7) == 7 and k(b"+1234567890123456789", 2, -1) == 1234567890123456789
    with pytest.raises(ValueError):
        Key("utf16")
    with pytest.raises(ValueError):
        _ = FixedWidth() + Key() + Key()
    with pytest.raises(TypeError):
        _ = VarLen() + Timestamp()


def test_native_loop_bad_verdict_commits_the_batches_before_and_never_yields(monkeypatch):
    """The fast stages return status -5 when the delivered batch's device verdict is bad
    (verify='deliver', torch_step.cpp verdict_bad): the loop commits what the user finished, then
    raises CorruptRecordException without yielding that batch.  A fake driver scripts the stage."""
    from collections import defaultdict

    import torchkafka_amd.loader.device_loader as dlm
    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset
    from torchkafka_amd.client.errors import CorruptRecordException

    class DS(KafkaDataset):
        schema = FixedWidth(torch.float32, (4,))

    dl = DeviceLoader(DS.placeholder(), 4, num_workers=1, device="cpu")
    assert dl.plan.fast_path and dl.verify == "deliver"

    class Drv:
        def __init__(self):
            self.calls = []

        def set_sync_commit(self, s):
            self.calls.append(("sync", s))

        def verify_delivered(self):
            raise AssertionError("the fast stages verify natively")

        def parse_error(self):
            return "RecordBatch CRC32C mismatch"

        def commit_pending(self):
            self.calls.append("commit")
            return 1

        def finish_delivered(self, stream):
            self.calls.append("finish")

        def finish_lockstep(self):
            self.calls.append("finish_lockstep")

        def drain_fenced(self, wait):
            pass

        def take_pending(self):
            return []

        def stats(self):
            st = defaultdict(int)
            st["commit_ns"] = []
            return st

        def committed(self):
            return []

        def delivered_positions(self):
            return []

        def delivered_batches(self):
            return 0

        def reset_stats(self):
            pass

    class Run:
        driver = Drv()
        closed = False

        def _check_workers_native(self):
            pass

        def close(self):
            Run.closed = True

    script = iter([(1, 0, "b0"), (1, 0, "b1"), (-5, 0, None), (1, 0, "never")])
    monkeypatch.setattr(dlm, "_stream_ptr", lambda device: 0)
    monkeypatch.setattr(DeviceLoader, "_fixed_stage", lambda self, drv, native_ac: (lambda: next(script)))
    got = []
    with pytest.raises(CorruptRecordException, match="CRC32C"):
        for b in dl._iterate_native(Run(), auto_commit=True):
            got.append(b)
    assert got == ["b0", "b1"]
    calls = Run.driver.calls
    assert calls.count("commit") == 1 and "finish_lockstep" not in calls  # b0/b1 committed, no clean end
    assert Run.closed
