"""gfx950 RecordBatch decode (DeviceLoader decode='device', csrc/hip/span_decode.hip) on the GPU.

The kernel reads record values straight out of the pinned broker logs, verifies the CRC32C of
every RecordBatch (kafka-python's check_crcs, reference kafka_dataset.py:156 loop) and casts the
values; every case is compared bit for bit with the host path (decode='host': workers CRC-check
and pack, the collate kernel casts), which tests/test_gpu_kernels.py pins to Tensor.to.
"""
import os
import random

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


def _run(broker, topic, DS, decode, bs, group, **kw):
    from torchkafka_amd import DeviceLoader, auto_commit

    dl = DeviceLoader(DS.placeholder(), bs, device="cuda:0", decode=decode,
                      worker_init_fn=DS.init_worker(topic, bootstrap_servers=broker.url, group_id=group,
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300), **kw)
    assert dl.plan.span == (decode == "device")
    xs = [x.clone() for x in auto_commit(dl)]
    torch.cuda.synchronize()
    return torch.cat(xs) if xs else None, dl


def _produce_random(broker, topic, n_parts, n_per_part, nbytes, rpb=16, seed=0, nulls=False):
    rng = random.Random(seed)
    for p in range(n_parts):
        vals, keys = [], []
        for o in range(n_per_part):
            vals.append(None if nulls and o % 5 == 2 else bytes(rng.getrandbits(8) for _ in range(nbytes)))
            keys.append(b"k" * rng.randrange(0, 9))  # shifts every value's alignment in the log
        for i in range(0, n_per_part, rpb):
            broker.produce(topic, vals[i:i + rpb], partition=p, keys=keys[i:i + rpb])


@pytest.mark.parametrize("shape,src,dst,norm,bs,rpb,workers", [
    ((256,), torch.float32, torch.bfloat16, False, 64, 64, 2),   # config 2's record shape
    ((256,), torch.float32, torch.float32, False, 50, 16, 1),    # batch boundaries inside RecordBatches
    ((13,), torch.float32, torch.float32, False, 33, 7, 2),      # 52-byte rows: partial 16-byte groups
    ((40,), torch.bfloat16, torch.float32, False, 32, 5, 1),     # 2-byte source elements
    ((48,), torch.uint8, torch.float16, False, 32, 9, 1),        # 1-byte source elements
    ((64,), torch.float32, torch.float8_e4m3fn, False, 40, 8, 2),
    ((64,), torch.float32, torch.bfloat16, True, 32, 16, 1),     # fused normalisation
    ((12000,), torch.float32, torch.bfloat16, False, 8, 4, 1),   # 192 KB RecordBatches: CRC chained over segments
    ((3,), torch.int32, torch.int64, False, 1000, 400, 1),       # tiny rows, many rows per segment
])
def test_device_decode_matches_host_path(broker, shape, src, dst, norm, bs, rpb, workers):
    numel = 1
    for d in shape:
        numel *= d
    esize = torch.empty((), dtype=src).element_size()
    n = 120 if numel < 1000 else 24
    broker.create_topic("t", 3)
    _produce_random(broker, "t", 3, n, numel * esize, rpb=rpb)
    from torchkafka_amd import FixedWidth

    DS = _dataset(FixedWidth(src, shape))
    normalize = (0.5, 2.0) if norm else None
    outs = {}
    for decode in ("host", "device"):
        outs[decode], _dl = _run(broker, "t", DS, decode, bs, f"g-{decode}", num_workers=workers, dtype=dst,
                                 normalize=normalize, in_order=True, coalesce=4)
        assert broker.committed_offsets(f"g-{decode}", "t") == {0: n, 1: n, 2: n}
    a, b = outs["host"], outs["device"]
    assert a.shape == b.shape == (3 * n, *shape)
    assert torch.equal(_bits(a), _bits(b))


def test_device_decode_values_and_commits(broker):
    """Known record contents (the synthetic f32 generator), several workers, exactly-once delivery."""
    from torchkafka_amd import FixedWidth

    broker.create_topic("t", 6)
    broker.fill("t", 300, "fixed_f32", size=32, records_per_batch=50)
    DS = _dataset(FixedWidth(torch.float32, (32,)))
    x, dl = _run(broker, "t", DS, "device", 64, "g", num_workers=3)
    seen = set()
    for row in x.cpu():
        o, p = int(row[0]), int(row[1])
        assert torch.equal(row, torch.tensor([synth_f32(p, o, j) for j in range(32)]))
        assert (p, o) not in seen
        seen.add((p, o))
    assert len(seen) == 1800
    assert broker.committed_offsets("g", "t") == {p: 300 for p in range(6)}
    assert dl.stats.log_bytes_registered > 0


def test_device_decode_skips_null_values_like_host(broker):
    from torchkafka_amd import FixedWidth

    broker.create_topic("t", 2)
    _produce_random(broker, "t", 2, 200, 64, rpb=11, nulls=True)
    DS = _dataset(FixedWidth(torch.float32, (16,)))
    a, _ = _run(broker, "t", DS, "host", 30, "gh", num_workers=1, in_order=True)
    b, _ = _run(broker, "t", DS, "device", 30, "gd", num_workers=1, in_order=True)
    assert a.shape == b.shape == (2 * 160, 16)
    assert torch.equal(_bits(a), _bits(b))
    assert broker.committed_offsets("gd", "t") == {0: 200, 1: 200}


def _corrupt(broker, pidx, pos):
    path = os.path.join(broker.native.dir, f"p{pidx:05d}.log")
    with open(path, "r+b") as f:
        f.seek(pos)
        b = f.read(1)
        f.seek(pos)
        f.write(bytes([b[0] ^ 0x5A]))


@pytest.mark.parametrize("size,rpb", [(64, 10), (12000, 4)])
def test_device_decode_crc_failure_raises_before_commit(broker, size, rpb):
    """A flipped value byte (the worker never reads values) is caught by the device CRC: the
    batch holding it is never committed and CorruptRecordException names its RecordBatch.
    size 12000 floats: the RecordBatch is split over segments, its CRC chained on the host."""
    from torchkafka_amd import FixedWidth
    from torchkafka_amd.client.errors import CorruptRecordException

    broker.create_topic("c", 1)
    n = 100 if size < 1000 else 24
    broker.fill("c", n, "fixed_f32", size=size, records_per_batch=rpb)
    pidx = broker.pidx("c", 0)
    # corrupt a value byte of the record at offset 4 * rpb + 1 (RecordBatch 4)
    row_bytes = size * 4
    bad_rb = 4
    log = broker.native.read_log(pidx, 0, broker.native.log_bytes(pidx))
    pos, k = 0, 0
    while k < bad_rb:
        pos += 12 + int.from_bytes(log[pos + 8:pos + 12], "big")
        k += 1
    _corrupt(broker, pidx, pos + 61 + 30 + row_bytes // 2)
    DS = _dataset(FixedWidth(torch.float32, (size,)))
    from torchkafka_amd import DeviceLoader, auto_commit

    bs = rpb
    dl = DeviceLoader(DS.placeholder(), bs, num_workers=1, device="cuda:0", decode="device", coalesce=1,
                      worker_init_fn=DS.init_worker("c", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    with pytest.raises(CorruptRecordException, match=f"offset {bad_rb * rpb} .*failed CRC check"):
        for _x in auto_commit(dl):
            torch.cuda.synchronize()
    committed = broker.committed_offsets("g", "c").get(0)
    assert committed is not None and committed <= bad_rb * rpb


@pytest.mark.parametrize("coalesce", [1, 8])
def test_verify_deliver_never_yields_a_corrupt_batch(broker, coalesce):
    """verify='deliver' (the default): a batch is handed out only after its device CRC verdict
    landed, so the loop body never sees the corrupt RecordBatch's records -- as kafka-python's
    check_crcs iterator raises before _process sees them (reference kafka_dataset.py:156-162).
    The batches before it are committed, it never is."""
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
    _corrupt(broker, pidx, pos + 61 + 30 + size * 2)
    DS = _dataset(FixedWidth(torch.float32, (size,)))
    dl = DeviceLoader(DS.placeholder(), rpb, num_workers=1, device="cuda:0", decode="device", coalesce=coalesce,
                      dtype=torch.float32,
                      worker_init_fn=DS.init_worker("c", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    assert dl.verify == "deliver"
    seen = []
    with pytest.raises(CorruptRecordException, match=f"offset {bad_rb * rpb} .*failed CRC check"):
        for x in auto_commit(dl):
            seen += x[:, 0].long().tolist()  # the user's step: reads every record of the batch
    assert seen == list(range(bad_rb * rpb)), (len(seen), seen[-3:])
    assert broker.committed_offsets("g", "c").get(0) == bad_rb * rpb


def test_device_decode_without_crc_checks(broker):
    """check_crcs=False: no verification anywhere (kafka-python semantics), only values are read."""
    from torchkafka_amd import DeviceLoader, FixedWidth, auto_commit

    broker.create_topic("t", 2)
    broker.fill("t", 200, "fixed_f32", size=32, records_per_batch=20)
    DS = _dataset(FixedWidth(torch.float32, (32,)))
    dl = DeviceLoader(DS.placeholder(), 64, num_workers=1, device="cuda:0", decode="device",
                      worker_init_fn=DS.init_worker("t", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300,
                                                    check_crcs=False))
    n = 0
    for x in auto_commit(dl):
        n += x.shape[0]
    assert n == 400 and broker.committed_offsets("g", "t") == {0: 200, 1: 200}


def test_device_decode_coalesced_batch_on_another_stream(broker):
    """Batches decoded ahead by a group launch, consumed on other streams, stay correct."""
    from torchkafka_amd import DeviceLoader, FixedWidth, auto_commit

    broker.create_topic("t", 4)
    broker.fill("t", 256, "fixed_f32", size=64, records_per_batch=32)
    DS = _dataset(FixedWidth(torch.float32, (64,)))
    dl = DeviceLoader(DS.placeholder(), 32, num_workers=2, device="cuda:0", decode="device", coalesce=8,
                      worker_init_fn=DS.init_worker("t", bootstrap_servers=broker.url, group_id="g",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=300))
    side = [torch.cuda.Stream(), torch.cuda.Stream()]
    copies = []
    it = iter(auto_commit(dl))
    k = 0
    while True:
        with torch.cuda.stream(side[k % 2]):
            try:
                x = next(it)
            except StopIteration:
                break
            copies.append(x.clone())
        k += 1
    torch.cuda.synchronize()
    rows = torch.cat(copies).cpu()
    assert rows.shape[0] == 1024
    for row in rows[::37]:
        o, p = int(row[0]), int(row[1])
        assert torch.equal(row, torch.tensor([synth_f32(p, o, j) for j in range(64)]))


@pytest.mark.parametrize("chunk_mib,chunks,rpb,size", [(1, 2, 16, 256), (1, 3, 4, 12000), (8, 4, 64, 256)])
def test_device_decode_through_hbm_mirror(broker, chunk_mib, chunks, rpb, size):
    """h2d='dma': the copy engines mirror the logs into HBM (log_mirror.h) and the kernel reads
    there; bit-exact with the host path, every byte mirrored once, buffers recycled safely."""
    from torchkafka_amd import FixedWidth, Tuning

    n = 600 if size < 1000 else 60
    broker.create_topic("t", 3)
    _produce_random(broker, "t", 3, n, size * 4, rpb=rpb)
    DS = _dataset(FixedWidth(torch.float32, (size,)))
    a, _ = _run(broker, "t", DS, "host", 32, "gh", num_workers=2, in_order=True)
    b, dl = _run(broker, "t", DS, "device", 32, "gm", num_workers=2, in_order=True, h2d="dma",
                 tuning=Tuning(mirror_chunk_mib=chunk_mib, mirror_chunks=chunks))
    assert dl.plan.mirror
    assert torch.equal(_bits(a), _bits(b))
    assert broker.committed_offsets("gm", "t") == {0: n, 1: n, 2: n}
    st = dl.stats_summary()
    assert st["mirror_copies"] > 0 and st["mirror_mib_copied"] > 0


def test_device_decode_generic_driver_path(broker):
    """return_info=True takes the driver's generic per-batch path: device-decoded batches arrive
    there too (KafkaBatch with watermarks), bit-exact with the host path."""
    from torchkafka_amd import FixedWidth

    broker.create_topic("t", 2)
    _produce_random(broker, "t", 2, 150, 64 * 4, rpb=10)
    DS = _dataset(FixedWidth(torch.float32, (64,)))
    from torchkafka_amd import DeviceLoader, auto_commit

    outs = {}
    for decode in ("host", "device"):
        dl = DeviceLoader(DS.placeholder(), 32, num_workers=1, device="cuda:0", decode=decode, return_info=True,
                          in_order=True, dtype=torch.bfloat16,
                          worker_init_fn=DS.init_worker("t", bootstrap_servers=broker.url, group_id=f"g{decode}",
                                                        auto_offset_reset="earliest", consumer_timeout_ms=300))
        bs = [b for b in auto_commit(dl)]
        assert all(b.watermarks for b in bs)
        outs[decode] = torch.cat([b.data.clone() for b in bs])
        assert broker.committed_offsets(f"g{decode}", "t") == {0: 150, 1: 150}
    assert torch.equal(_bits(outs["host"]), _bits(outs["device"]))


@pytest.mark.parametrize("src,dst,lens,nulls,long_every,opts", [
    (torch.int32, torch.int64, (0, 300), 0, 0, {}),                                   # token ids
    (torch.int32, torch.int32, (1, 60), 7, 11, {"return_mask": True, "pad_value": -1}),  # worker-copied long rows
    (torch.uint8, torch.float16, (0, 90), 0, 0, {"pad_to": 128}),
    (torch.float16, torch.bfloat16, (0, 40), 5, 0, {"pad_multiple": 16}),  # 2-byte elements, any bits
])
def test_var_span_matches_host_path(broker, src, dst, lens, nulls, long_every, opts):
    """VarLen records decoded on the device from the logs (varlen_span_kernel) == the host CSR
    pack + varlen collate kernel, bit for bit (lengths, padding and masks included)."""
    import struct

    from torchkafka_amd import DeviceLoader, VarLen, auto_commit
    from torchkafka_amd.ops.native import core

    esize = torch.empty((), dtype=src).element_size()
    fmt = {1: "B", 2: "H", 4: "i"}[esize]
    rng = random.Random(esize * 7 + lens[1])
    broker.create_topic("v", 2)
    for p in range(2):
        vals = []
        for i in range(180):
            if nulls and i % nulls == 3:
                vals.append(None)
                continue
            k = rng.randint(*lens)
            if long_every and i % long_every == 2:
                k = core().VAR_SPAN_ROW_MAX // esize + rng.randint(1, 300)
            lo, hi = (0, (1 << (8 * esize)) - 1) if fmt in "BH" else (-(1 << 31), (1 << 31) - 1)
            vals.append(struct.pack(f"<{k}{fmt}", *[rng.randint(lo, hi) for _ in range(k)]))
        for i in range(0, len(vals), 13):
            broker.produce("v", vals[i:i + 13], partition=p)
    DS = _dataset(VarLen(src))
    outs = {}
    for decode in ("host", "device"):
        dl = DeviceLoader(DS.placeholder(), 32, num_workers=2, device="cuda:0", decode=decode, dtype=dst,
                          in_order=True, coalesce=4,
                          worker_init_fn=DS.init_worker("v", bootstrap_servers=broker.url, group_id=f"g{decode}",
                                                        auto_offset_reset="earliest", consumer_timeout_ms=300),
                          **opts)
        assert dl.plan.var_span == (decode == "device")
        outs[decode] = [tuple(t.clone() for t in b) for b in auto_commit(dl)]
        assert broker.committed_offsets(f"g{decode}", "v") == {0: 180, 1: 180}
    a, b = outs["host"], outs["device"]
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert len(x) == len(y)
        for u, v in zip(x, y):
            assert u.shape == v.shape and u.dtype == v.dtype
            assert torch.equal(_bits(u) if u.is_floating_point() else u, _bits(v) if v.is_floating_point() else v)


def test_hbm_mirror_copies_across_pin_pieces(broker):
    """A log longer than the driver's 64 MiB pin pieces: the mirror splits its copies at the piece
    boundaries (a DMA source must lie in one registration); values intact across them."""
    import os
    import uuid

    from torchkafka_amd import FixedWidth, Tuning
    from torchkafka_amd.broker import SyntheticBroker

    big = SyntheticBroker.create(f"shm://tkbig-{os.getpid()}-{uuid.uuid4().hex[:6]}", log_capacity=256 << 20)
    try:
        big.create_topic("t", 1)
        big.fill("t", 90_000, "fixed_f32", size=256, records_per_batch=64)  # ~93 MB: two pin pieces
        DS = _dataset(FixedWidth(torch.float32, (256,)))
        b, dl = _run(big, "t", DS, "device", 256, "gm", num_workers=1, in_order=True, h2d="dma",
                     tuning=Tuning(mirror_chunk_mib=8, mirror_chunks=4))
        assert dl.plan.mirror and b.shape == (90_000, 256)
        assert torch.equal(b[:, 0], torch.arange(90_000, dtype=torch.float32, device=b.device))
        for o in (0, 65_000, 89_999):
            assert torch.equal(b[o].cpu(), torch.tensor([synth_f32(0, o, j) for j in range(256)]))
    finally:
        big.destroy()


@pytest.fixture
def big_broker():
    """A broker whose partition logs hold a few hundred MiB (the shared fixture's hold 64 MiB)."""
    import uuid

    from torchkafka_amd.broker import SyntheticBroker

    b = SyntheticBroker.create(f"shm://tkbig-{os.getpid()}-{uuid.uuid4().hex[:8]}", log_capacity=1 << 30,
                               index_capacity=1 << 18)
    try:
        yield b
    finally:
        b.destroy()


def test_mirror_pins_only_up_to_the_chunk_holding_the_written_end(big_broker):
    """h2d='dma' over a pre-filled log: the mirror's reads never make LogPins register past the
    64 MiB piece that holds each partition's written end (the round-3 look-ahead registered up to
    128 MiB of unwritten log on the launch thread)."""
    from torchkafka_amd import FixedWidth

    chunk = 64 << 20
    big_broker.create_topic("t", 2)
    big_broker.fill("t", 20000, "fixed_f32", size=1024, records_per_batch=32)  # ~82 MB per partition
    DS = _dataset(FixedWidth(torch.float32, (1024,)))
    written = [big_broker.native.log_bytes(big_broker.pidx("t", p)) for p in range(2)]
    x, dl = _run(big_broker, "t", DS, "device", 256, "gp", num_workers=2, h2d="dma")
    assert dl.plan.mirror and x.shape == (40000, 1024)
    want = sum((w + chunk - 1) // chunk * chunk for w in written)
    assert dl.stats.log_bytes_registered <= want, (dl.stats.log_bytes_registered, want, written)


def test_growing_log_is_pinned_off_the_launch_thread(big_broker):
    """A live tail: records keep arriving while the loader decodes them from the pinned logs.  The
    pin thread registers each new 64 MiB piece as the written end reaches it; every record arrives
    exactly once and the launch thread's wait for pinning stays a small part of the run."""
    import threading
    import time

    from torchkafka_amd import DeviceLoader, FixedWidth, auto_commit

    big_broker.create_topic("t", 2)
    big_broker.fill("t", 2000, "fixed_f32", size=1024, records_per_batch=50)
    DS = _dataset(FixedWidth(torch.float32, (1024,)))
    stop = threading.Event()
    rounds = 60

    def produce():  # ~8 MB per partition per round: the logs cross several 64 MiB pieces
        for _ in range(rounds):
            big_broker.fill("t", 2000, "fixed_f32", size=1024, records_per_batch=50)
            time.sleep(0.01)
        stop.set()

    th = threading.Thread(target=produce)
    th.start()
    dl = DeviceLoader(DS.placeholder(), 256, num_workers=2, device="cuda:0", dtype=torch.float32,
                      worker_init_fn=DS.init_worker("t", bootstrap_servers=big_broker.url, group_id="gl",
                                                    auto_offset_reset="earliest", consumer_timeout_ms=1500))
    t0 = time.perf_counter()
    seen = 0
    last = {}
    for x in auto_commit(dl):
        rows = x[:, :2].long().cpu()
        seen += rows.shape[0]
        for p in (0, 1):
            o = rows[rows[:, 1] == p][:, 0]
            if o.numel():
                assert int(o[0]) == last.get(p, -1) + 1  # in order, nothing skipped or repeated
                last[p] = int(o[-1])
    el = time.perf_counter() - t0
    th.join()
    st = dl.stats_summary()
    total = 2000 * (rounds + 1)
    assert seen == 2 * total and last == {0: total - 1, 1: total - 1}
    assert st["log_pin_ms"] > 0 and dl.stats.log_bytes_registered >= 2 * (total * 4096 // (64 << 20)) * (64 << 20)
    assert st["log_pin_wait_ms"] < 0.25 * el * 1e3, (st["log_pin_wait_ms"], el)
