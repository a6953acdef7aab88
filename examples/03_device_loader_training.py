#!/usr/bin/env python3
"""MI355X device path: Kafka records -> pinned ring -> gfx950 collate (bf16, fused normalisation)
-> a training step, committing each batch after the step (exact offsets), with the committed
offsets saved next to the model checkpoint and restored on restart.

Single GPU:     python examples/03_device_loader_training.py
DDP (8 GPUs):   python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
                    examples/03_device_loader_training.py
Each rank consumes its own partitions (static sharding) and the ranks step in lockstep over RCCL,
so they stop together and only commit batches every rank finished.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from torchkafka import DeviceLoader, FixedWidth, KafkaDataset, auto_commit  # noqa: E402
from torchkafka_amd.broker import SyntheticBroker  # noqa: E402


class Features(KafkaDataset):
    schema = FixedWidth(torch.float32, (256,))  # 1 KiB records decoded natively in the workers


def main():
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    url = f"shm://example3-{os.getppid() if world > 1 else os.getpid()}"
    broker = SyntheticBroker.create(url)
    broker.create_topic("features", 8 * world)
    mine = [p for p in range(8 * world) if p % world == rank]
    broker.fill("features", 2048, "fixed_f32", size=256, partitions=mine)
    if world > 1:
        dist.init_process_group("nccl")  # the loader forks its workers before HIP is initialised
    device = torch.device("cuda", local)
    loader = DeviceLoader(Features.placeholder(), 256, num_workers=4, device=device, dtype=torch.bfloat16,
                          normalize=(0.0, 100.0),
                          worker_init_fn=Features.init_worker("features", bootstrap_servers=url, group_id="train",
                                                              auto_offset_reset="earliest", consumer_timeout_ms=500))
    ckpt = f"/tmp/example3-offsets-rank{rank}.json"
    if os.path.exists(ckpt):  # resume where the last checkpoint's offsets say
        loader.load_state_dict(json.load(open(ckpt)))
    model = torch.nn.Linear(256, 16).to(device=device, dtype=torch.bfloat16)
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)
    steps = 0
    for x in auto_commit(loader):  # x: [256, 256] bf16 on this rank's GPU
        loss = model(x).float().pow(2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        steps += 1
        if steps % 20 == 0:
            json.dump(loader.state_dict(), open(ckpt, "w"))  # committed offsets = data checkpoint
    torch.cuda.synchronize()
    print(f"[rank {rank}] {steps} steps; committed {loader.state_dict()['offsets']}")
    os.remove(ckpt) if os.path.exists(ckpt) else None
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        broker.destroy()


if __name__ == "__main__":
    main()
