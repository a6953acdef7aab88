#!/usr/bin/env python3
"""DDP training fed from Kafka on the MI355X device path, with a checkpoint that resumes exactly once.

Kafka records -> workers -> gfx950 decode (bf16, fused normalisation) -> DistributedDataParallel step
-> the batch is committed after the step (exact offsets).  Every ``--ckpt-every`` steps rank 0 writes
ONE checkpoint: the model and optimiser state beside ``loader.state_dict(global_step=True)`` -- the
delivered positions of EVERY rank at the same agreed global step (each rank consumes its own
partitions, so a per-rank ``state_dict()`` taken at different moments would not describe one step of
the job).  A restart loads both: the model continues from step S and every rank's workers start right
after the records of step S -- no record trained twice, none skipped.

The reference checkpoints nothing itself: its committed offsets are the checkpoint and close() never
commits (/root/reference/src/kafka_dataset.py:85-91); its multi-worker usage is README.md:103-132.

    python examples/03_device_loader_training.py                       # one GPU
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        examples/03_device_loader_training.py                          # DDP, 8 GPUs (RCCL gradients)
    ... --device cpu                                                   # gloo, no GPU (tests/test_examples.py)

The ranks step in lockstep (the node-local shared-memory agreement on one host), so a rank that runs
out of records stops every rank at the same step instead of leaving DDP's all-reduce hanging.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.nn.parallel import DistributedDataParallel as DDP  # noqa: E402

from torchkafka import DeviceLoader, FixedWidth, KafkaDataset, auto_commit  # noqa: E402
from torchkafka_amd.broker import SyntheticBroker  # noqa: E402
from torchkafka_amd.broker.synthetic import open_broker  # noqa: E402


class Features(KafkaDataset):
    schema = FixedWidth(torch.float32, (256,))  # 1 KiB records: column 0 = offset, 1 = partition


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--broker", default=None, help="an existing broker URL (default: a fresh synthetic one)")
    ap.add_argument("--records", type=int, default=2048, help="records per partition of a fresh broker")
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--ckpt-dir", default="/tmp/example3-ckpt")
    ap.add_argument("--ckpt-every", type=int, default=20)
    ap.add_argument("--stop-after", type=int, default=None,
                    help="leave after this global step, right after its checkpoint (a preemption)")
    ap.add_argument("--trace-dir", default=None, help="write the (partition, offset) of every trained record")
    return ap.parse_args()


def main():
    a = parse()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    on_gpu = a.device == "cuda"
    device = torch.device("cuda", local) if on_gpu else torch.device("cpu")
    # the process group first (no GPU touched: RCCL makes its communicator at the first collective,
    # after the loader forked its workers)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29513")
    dist.init_process_group("nccl" if on_gpu else "gloo", rank=rank, world_size=world)
    own = a.broker is None
    url = a.broker or f"shm://example3-{os.environ['MASTER_PORT']}"
    if own and rank == 0:
        b = SyntheticBroker.create(url)
        b.create_topic("features", 8 * world)
        b.fill("features", a.records, "fixed_f32", size=256)
    dist.barrier()
    broker = open_broker(url)

    # bf16 with a fused normalisation; a traced run keeps float32 so the offset column stays exact
    fmt = dict(dtype=torch.float32) if a.trace_dir else dict(dtype=torch.bfloat16, normalize=(0.0, 100.0))
    loader = DeviceLoader(Features.placeholder(), a.batch_size, num_workers=2 if not on_gpu else 4, device=device,
                          **fmt,
                          worker_init_fn=Features.init_worker("features", bootstrap_servers=url, group_id="train",
                                                              auto_offset_reset="earliest", consumer_timeout_ms=500))
    model = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.GELU(), torch.nn.Linear(512, 16))
    model = model.to(device=device, dtype=torch.bfloat16)
    ddp = DDP(model, device_ids=[local] if on_gpu else None)
    opt = torch.optim.SGD(ddp.parameters(), lr=1e-3)

    ckpt = os.path.join(a.ckpt_dir, "latest.pt")
    step = 0
    if os.path.exists(ckpt):  # every rank reads the one checkpoint rank 0 wrote
        state = torch.load(ckpt, map_location="cpu", weights_only=True)
        model.load_state_dict(state["model"])
        opt.load_state_dict(state["opt"])
        step = int(state["step"])
        loader.load_state_dict(json.loads(state["data"]))  # commits every rank's positions of step S
    first_step = step

    trace = []
    stopped = False
    for x in auto_commit(loader):  # x: [batch, 256] bf16, this rank's partitions only
        if a.trace_dir:
            trace += [(p, o) for o, p in x[:, :2].long().tolist()]  # fixed_f32: offset, partition
        loss = ddp(x.to(torch.bfloat16)).float().pow(2).mean()
        opt.zero_grad(set_to_none=True)
        loss.backward()  # DDP all-reduces the gradients (RCCL on GPUs)
        opt.step()
        step += 1
        if step % a.ckpt_every == 0 or step == a.stop_after:
            data = loader.state_dict(global_step=True)  # a collective: every rank, same step
            if rank == 0:
                os.makedirs(a.ckpt_dir, exist_ok=True)
                tmp = ckpt + ".tmp"
                torch.save({"model": model.state_dict(), "opt": opt.state_dict(), "step": step,
                            "data": json.dumps(data)}, tmp)
                os.replace(tmp, ckpt)
        if step == a.stop_after:
            stopped = True
            break  # the batch of this step is in the checkpoint: never committed twice, never lost
    if on_gpu:
        torch.cuda.synchronize(device)
    loader.close()
    if a.trace_dir:
        os.makedirs(a.trace_dir, exist_ok=True)
        with open(os.path.join(a.trace_dir, f"rank{rank}-from{first_step}.json"), "w") as f:
            json.dump(trace, f)
    print(f"[rank {rank}] steps {first_step}..{step}{' (stopped)' if stopped else ''}; "
          f"committed {broker.committed_offsets('train', 'features')}", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if own and rank == 0 and not stopped:
        broker.destroy()


if __name__ == "__main__":
    main()
