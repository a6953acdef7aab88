"""A Kafka cluster feeding the gfx950 decode path (KafkaBridge -> replica logs -> span_decode).

The native replicator receives Fetch responses into the tails of local partition logs while the
loader pins those logs and decodes batches from them on the device (CRC32C + cast,
csrc/hip/span_decode.hip).  The cluster is `KafkaWireServer` over a synthetic broker (no Kafka
cluster exists on the box); results are compared bit for bit with the host decode path, and the
cluster's committed offsets are checked after close().
"""
import os
import time
import uuid

import pytest
import torch

from conftest import synth_f32

pytestmark = pytest.mark.gpu


def _loader(DS, url, decode, bs=64):
    from torchkafka_amd import DeviceLoader

    return DeviceLoader(DS.placeholder(), bs, num_workers=2, device="cuda:0", decode=decode, dtype=torch.float32,
                        worker_init_fn=DS.init_worker("t", bootstrap_servers=url, group_id=f"trainer-{decode}",
                                                      auto_offset_reset="earliest", consumer_timeout_ms=400))


@pytest.mark.parametrize("live", [False, True])
def test_device_decode_from_a_replicated_cluster(broker, live):
    from torchkafka_amd import FixedWidth, KafkaDataset, auto_commit
    from torchkafka_amd.broker import KafkaBridge, KafkaWireServer

    class Rows(KafkaDataset):
        schema = FixedWidth(torch.float32, (256,))

    broker.create_topic("t", 4)
    broker.fill("t", 600 if live else 1200, "fixed_f32", size=256, records_per_batch=64)
    out = {}
    with KafkaWireServer(broker) as srv:
        for decode in ("device", "host"):
            br = KafkaBridge(srv.address, "t", group_id=f"trainer-{decode}",
                             url=f"shm://tkgbr-{os.getpid()}-{uuid.uuid4().hex[:6]}", log_capacity=256 << 20)
            try:
                if not live:
                    assert br.wait_caught_up(20)
                dl = _loader(Rows, br.url, decode)
                assert dl.plan.span == (decode == "device")
                xs = []
                for i, x in enumerate(auto_commit(dl)):
                    xs.append(x.clone())
                    if live and decode == "device" and i == 3:
                        # the cluster keeps producing while the replica is being decoded from
                        broker.fill("t", 600, "fixed_f32", size=256, records_per_batch=64)
                    if live and decode == "device" and i == 4:
                        time.sleep(0.2)
                torch.cuda.synchronize()
                out[decode] = torch.cat(xs)
            finally:
                br.close()
            assert broker.committed_offsets(f"trainer-{decode}", "t") == {p: 1200 for p in range(4)}
    d, h = out["device"], out["host"]
    assert d.shape == h.shape == (4800, 256)
    key = lambda t: (t[:, 1].float() * 1e6 + t[:, 0].float()).argsort()  # noqa: E731 -- (partition, offset) order
    assert torch.equal(d[key(d)].view(torch.int32), h[key(h)].view(torch.int32))


def test_long_stream_unpins_and_releases_consumed_log(broker):
    """A replica stream longer than the driver's 64 MiB pin chunks: committed ranges are unpinned
    by the driver and punched out of the replica files by the replicator, and decoding goes on."""
    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
    from torchkafka_amd.broker import KafkaBridge, KafkaWireServer, SyntheticBroker

    class Rows(KafkaDataset):
        schema = FixedWidth(torch.float32, (256,))

    src = SyntheticBroker.create(f"shm://tkgsrc-{os.getpid()}-{uuid.uuid4().hex[:6]}", log_capacity=512 << 20)
    try:
        src.create_topic("t", 1)
        src.fill("t", 160_000, "fixed_f32", size=256, records_per_batch=64)  # ~165 MB
        with KafkaWireServer(src) as srv:
            br = KafkaBridge(srv.address, "t", group_id="g", url=f"shm://tkgbr-{os.getpid()}-{uuid.uuid4().hex[:6]}",
                             log_capacity=512 << 20, max_lag_bytes=96 << 20, release_bytes=16 << 20,
                             release_step=64 << 20, ring_bytes=0)  # a linear replica with release
            try:
                dl = DeviceLoader(Rows.placeholder(), 256, num_workers=1, device="cuda:0", dtype=torch.float32,
                                  worker_init_fn=Rows.init_worker("t", bootstrap_servers=br.url, group_id="g",
                                                                  auto_offset_reset="earliest",
                                                                  consumer_timeout_ms=1000))
                assert dl.plan.span
                n, last = 0, -1
                for x in auto_commit(dl):
                    offs = x[:, 0]
                    assert int(offs[0].item()) == last + 1  # one partition, in order
                    last = int(offs[-1].item())
                    n += x.shape[0]
                torch.cuda.synchronize()
                assert n == 160_000 and last == 159_999
                assert dl.stats.log_bytes_unpinned >= 64 << 20
                released = br.stats()[0]["released"]
                assert released >= 64 << 20, br.stats()
            finally:
                br.close()
        assert src.committed("g", "t", 0) == 160_000
    finally:
        src.destroy()


def test_ring_replica_long_stream_device_decode(broker):
    """The default replica: a 32 MiB ring per partition carries a ~165 MB stream.  Segments are read
    zero-copy from the pinned ring while the replicator writes over committed batches; values and
    order exact, every offset committed to the cluster."""
    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
    from torchkafka_amd.broker import KafkaBridge, NativeWireServer, SyntheticBroker

    class Rows(KafkaDataset):
        schema = FixedWidth(torch.float32, (256,))

    src = SyntheticBroker.create(f"shm://tkgsrc-{os.getpid()}-{uuid.uuid4().hex[:6]}", log_capacity=512 << 20)
    try:
        src.create_topic("t", 1)
        src.fill("t", 160_000, "fixed_f32", size=256, records_per_batch=64)
        with NativeWireServer(src) as srv:
            br = KafkaBridge(srv.address, "t", group_id="g", url=f"shm://tkgbr-{os.getpid()}-{uuid.uuid4().hex[:6]}",
                             ring_bytes=32 << 20, log_capacity=64 << 20, max_partition_fetch_bytes=4 << 20)
            try:
                dl = DeviceLoader(Rows.placeholder(), 256, num_workers=1, device="cuda:0", dtype=torch.float32,
                                  worker_init_fn=Rows.init_worker("t", bootstrap_servers=br.url, group_id="g",
                                                                  auto_offset_reset="earliest",
                                                                  consumer_timeout_ms=1500))
                assert dl.plan.span
                n, last = 0, -1
                for x in auto_commit(dl):
                    assert int(x[0, 0].item()) == last + 1
                    if n % 64000 == 0:
                        o = int(x[7, 0].item())
                        assert torch.equal(x[7].cpu(), torch.tensor([synth_f32(0, o, j) for j in range(256)]))
                    last = int(x[-1, 0].item())
                    n += x.shape[0]
                torch.cuda.synchronize()
                dl.close()
                assert n == 160_000 and last == 159_999
                assert br.local.native.first_batch(br.local.pidx("t", 0)) > 0
            finally:
                br.close()
        assert src.committed("g", "t", 0) == 160_000
    finally:
        src.destroy()


@pytest.mark.parametrize("schema_kind", ["fixed", "varlen"])
def test_sync_commit_on_the_device_path(broker, schema_kind):
    """commit='sync' through the native step driver: before batch k+1 is handed out, batch k's
    device verdict landed and the coordinator answered its OffsetCommit (bridge='auto')."""
    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, VarLen, auto_commit
    from torchkafka_amd.broker import NativeWireServer

    class Rows(KafkaDataset):
        schema = FixedWidth(torch.float32, (64,)) if schema_kind == "fixed" else VarLen(torch.float32, max_len=64)

    broker.create_topic("t", 4)
    if schema_kind == "fixed":
        broker.fill("t", 400, "fixed_f32", size=64, records_per_batch=20)
    else:
        broker.fill("t", 400, "varlen_f32", size=8, max_size=64, records_per_batch=20)
    with NativeWireServer(broker, profile="kafka4") as srv:
        dl = DeviceLoader(Rows.placeholder(), 32, num_workers=2, device="cuda:0", commit="sync", dtype=torch.float32,
                          worker_init_fn=Rows.init_worker("t", bootstrap_servers=srv.address, group_id="sync",
                                                          auto_offset_reset="earliest", consumer_timeout_ms=500))
        assert dl._bridges, "bridge='auto' mirrors the cluster"
        n, batches = 0, 0
        for x in auto_commit(dl):
            got = broker.committed_offsets("sync", "t")
            if batches >= 1:  # what the previous batches covered is at the coordinator already
                assert sum(v or 0 for v in got.values()) >= n, (got, n)
            rows = x[0] if isinstance(x, tuple) else x
            n += rows.shape[0]
            batches += 1
        st = dl.stats_summary()
        dl.close()
    assert n == 1600 and broker.committed_offsets("sync", "t") == {p: 400 for p in range(4)}
    assert st["sync_commits"] >= batches - 1 and st["commit_failures"] == 0
