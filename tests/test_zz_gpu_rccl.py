"""RCCL (torch 'nccl' backend) lockstep on one GPU -- runs last in the GPU session."""
import pytest

pytestmark = pytest.mark.gpu


def test_lockstep_rccl_world1():
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import nccl_probe

    nccl_probe.main()


def test_native_rccl_lockstep_driver_world1(broker):
    """The driver's pipelined lockstep over a real RCCL communicator (world 1), all depths."""
    import os

    import torch
    import torch.distributed as dist

    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit

    class Vec(KafkaDataset):
        schema = FixedWidth(torch.float32, (8,))

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = "29541"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        broker.create_topic("t", 2)
        broker.fill("t", 95, "fixed_f32", size=8)
        for depth in (0, 1, 3):
            dl = DeviceLoader(Vec.placeholder(), 20, num_workers=2, device="cuda:0", lockstep="rccl",
                              lockstep_depth=depth,
                              worker_init_fn=Vec.init_worker("t", bootstrap_servers=broker.url, group_id=f"g{depth}",
                                                             auto_offset_reset="earliest", consumer_timeout_ms=300))
            n = sum(x.shape[0] for x in auto_commit(dl))
            assert n == 190
            assert broker.committed_offsets(f"g{depth}", "t") == {0: 95, 1: 95}
    finally:
        dist.destroy_process_group()


def test_rccl_lockstep_transport_failure_detection_plumbing():
    """The native transport's bounded wait (failure detection) at world size 1: results come back,
    the timeout is settable and nothing is aborted.  (A dead peer cannot be staged on a 1-GPU box;
    the timeout/abort path is exercised by multi-GPU runs.)"""
    import os

    import torch

    from torchkafka_amd.ops.native import hip

    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    # the agreement's four words reach RCCL through tiny copy kernels (default), as host-mapped
    # buffers handed to RCCL itself, by hipMemcpyAsync (A/B), or the three operations captured into
    # one HIP graph per slot
    for mode in ("kernel", "host", "copy", "graph"):
        os.environ["TORCHKAFKA_RCCL_WORDS"] = mode
        try:
            uid = hip().RcclLockstep.unique_id(lib)
            ls = hip().RcclLockstep(lib, uid, 0, 1, 0, 3)
        finally:
            del os.environ["TORCHKAFKA_RCCL_WORDS"]
        assert ls.words_mode == mode
        assert ls.timeout_ms == 600000
        ls.set_timeout_ms(2000)
        assert ls.timeout_ms == 2000
        for i in range(10):
            assert ls.allreduce_min(i, -i, 7, 2 - i % 3) == (i, -i, 7, 2 - i % 3)
        assert not ls.aborted
        del ls


def test_native_rccl_lockstep_sync_commit_world1(broker):
    """commit='sync' through the RCCL lockstep (world 1, lockstep='rccl'): one agreement per step
    makes batch k committable before batch k+1 is handed out, and k's offsets are stored then."""
    import os

    import torch
    import torch.distributed as dist

    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
    from test_gpu_sync_lockstep import batch_ends

    class Vec(KafkaDataset):
        schema = FixedWidth(torch.float32, (8,))

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = "29543"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        broker.create_topic("t", 2)
        broker.fill("t", 200, "fixed_f32", size=8, records_per_batch=10)
        dl = DeviceLoader(Vec.placeholder(), 20, num_workers=2, device="cuda:0", lockstep="rccl", commit="sync",
                          dtype=torch.float32,
                          worker_init_fn=Vec.init_worker("t", bootstrap_servers=broker.url, group_id="gsync",
                                                         auto_offset_reset="earliest", consumer_timeout_ms=300))
        want, steps, bad = {}, 0, []
        for x in auto_commit(dl):
            if steps:
                got = {p: o for p, o in broker.committed_offsets("gsync", "t").items() if p in want}
                if got != want:
                    bad.append((steps, got, dict(want)))
            for p, e in batch_ends(x).items():
                want[p] = max(want.get(p, 0), e)
            steps += 1
        st = dl.stats_summary()
        info = dict(dl.lockstep_info)
        dl.close()
        assert info.get("transport") == "rccl"
        assert steps == 20 and bad == []
        assert st["commits"] >= steps - 1
        assert broker.committed_offsets("gsync", "t") == {0: 200, 1: 200}
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("transport", ["shm", "rccl"])
def test_rehearsed_ddp_stream_plan_fits_the_hardware_queues(broker, transport):
    """VERDICT r5 do-this 1: the N = 8 stream layout, rehearsed on one GPU (a world-1 nccl group
    whose all-reduce made torch's own RCCL communicator and stream, as a DDP job's gradient
    all-reduce does), fits the process's 4 hardware queues: the decode streams give way to torch's
    NCCL stream and the lockstep's, so no decode kernel shares a queue with a collective."""
    import os

    import torch
    import torch.distributed as dist

    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit

    class Vec(KafkaDataset):
        schema = FixedWidth(torch.float32, (64,))

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = "29547" if transport == "shm" else "29549"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    os.environ["TORCHKAFKA_TORCH_NCCL_ACTIVE"] = "1"
    try:
        dist.all_reduce(torch.ones(1, device="cuda:0"))
        torch.cuda.synchronize()
        broker.create_topic("t", 2)
        broker.fill("t", 400, "fixed_f32", size=64)
        dl = DeviceLoader(Vec.placeholder(), 20, num_workers=2, device="cuda:0", lockstep=transport,
                          worker_init_fn=Vec.init_worker("t", bootstrap_servers=broker.url, group_id=f"sp{transport}",
                                                         auto_offset_reset="earliest", consumer_timeout_ms=300))
        n = sum(x.shape[0] for x in auto_commit(dl))
        plan = dict(dl.lockstep_info["streams"])
        dl.close()
        assert n == 800
        assert plan["torch_nccl"] == 1 and plan["decode"] >= 1, plan
        assert plan["rccl_lockstep"] == (1 if transport == "rccl" else 0), plan
        assert not plan["shared"] and plan["total"] <= plan["hw_queues"], plan
    finally:
        os.environ.pop("TORCHKAFKA_TORCH_NCCL_ACTIVE", None)
        dist.destroy_process_group()
