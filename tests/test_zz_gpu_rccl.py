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
            dl = DeviceLoader(Vec.placeholder(), 20, num_workers=2, device="cuda:0", lockstep="always",
                              lockstep_depth=depth,
                              worker_init_fn=Vec.init_worker("t", bootstrap_servers=broker.url, group_id=f"g{depth}",
                                                             auto_offset_reset="earliest", consumer_timeout_ms=300))
            n = sum(x.shape[0] for x in auto_commit(dl))
            assert n == 190
            assert broker.committed_offsets(f"g{depth}", "t") == {0: 95, 1: 95}
    finally:
        dist.destroy_process_group()
