"""RCCL (torch 'nccl' backend) probe for the lockstep path, world size 1 on one GPU.

Prints a line per step (flushed) so a hang shows exactly where it stopped.
Run under a time limit: ``timeout -k 5 90 python tools/nccl_probe.py``.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def say(*a):
    print(f"[{time.strftime('%T')}]", *a, flush=True)


def main():
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
    say("init_process_group nccl")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    say("all_reduce on current stream")
    t = torch.ones(3, dtype=torch.int64, device="cuda:0")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    torch.cuda.synchronize()
    say("ok", t.tolist())
    from torchkafka_amd.parallel import Lockstep

    say("Lockstep side-stream agree")
    lk = Lockstep(device=torch.device("cuda", 0))
    assert lk.agree(True, 0)
    assert not lk.agree(False, 1)
    t0 = time.perf_counter()
    for i in range(200):
        lk.agree(True, i)
    say(f"lockstep agree: {(time.perf_counter() - t0) / 200 * 1e6:.1f} us/step (world 1)")
    lk.barrier()
    dist.destroy_process_group()
    say("done")


if __name__ == "__main__":
    main()
