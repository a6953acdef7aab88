#!/usr/bin/env python3
"""Round trip of one lockstep agreement over RCCL at world 1 (RcclLockstep.allreduce_min: the four
words in, all-reduce(MIN), out), idle and beside GPU load on other streams, per words mode.

The loader issues one agreement per credit grant and waits for it when its credits run out; the
round trip is what the lockstep costs a step when it is longer than the steps the credits cover.
Usage: python tools/probes/rccl_rtt.py [--iters 2000]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(len(xs) * q))], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    args = ap.parse_args()
    from torchkafka_amd.ops.native import hip

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    out = {}
    # the loader load: config 2 stepping on a thread of its own (its steps release the GIL)
    import threading
    import uuid

    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    class Rec(KafkaDataset):
        schema = FixedWidth(torch.float32, (256,))

    url = f"shm://tkrtt-{os.getpid()}-{uuid.uuid4().hex[:6]}"
    broker = SyntheticBroker.create(url, log_capacity=1 << 30, index_capacity=1 << 20)
    broker.create_topic("t", 8)
    broker.fill("t", 600000, "fixed_f32", size=256, records_per_batch=64, threads=8)
    stop = threading.Event()
    loader_batches = [0]

    def run_loader(group):
        dl = DeviceLoader(Rec.placeholder(), 256, num_workers=4, device=dev, dtype=torch.bfloat16,
                          worker_init_fn=Rec.init_worker("t", bootstrap_servers=url, group_id=group,
                                                         auto_offset_reset="earliest", consumer_timeout_ms=2000))
        it = iter(auto_commit(dl))
        for _ in it:
            loader_batches[0] += 1
            if stop.is_set():
                break
        it.close()
        dl.close()

    side = torch.cuda.Stream(dev)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    small = torch.randn(4 << 20, device=dev)
    for mode in ("kernel", "host", "copy"):
        os.environ["TORCHKAFKA_RCCL_WORDS"] = mode
        uid = hip().RcclLockstep.unique_id(lib)
        ls = hip().RcclLockstep(lib, uid, 0, 1, 0, 3)
        del os.environ["TORCHKAFKA_RCCL_WORDS"]
        for _ in range(50):
            ls.allreduce_min(1, 2, 3, 4)
        res = {}
        for load in ("idle", "elementwise", "gemm", "loader"):
            ts = []
            th = None
            if load == "loader":
                stop.clear()
                th = threading.Thread(target=run_loader, args=(f"g-{mode}",))
                th.start()
                time.sleep(1.0)
            for i in range(args.iters):
                if load != "idle" and i % 8 == 0:
                    with torch.cuda.stream(side):
                        for _ in range(4):
                            if load == "gemm":
                                torch.matmul(a, a)
                            else:
                                small.mul_(1.0001)
                t0 = time.perf_counter_ns()
                ls.allreduce_min(i, -i, 7, 2)
                ts.append((time.perf_counter_ns() - t0) / 1e3)
            if th is not None:
                stop.set()
                th.join()
            torch.cuda.synchronize()
            res[load] = {"p50_us": pct(ts, 0.5), "p90_us": pct(ts, 0.9), "p99_us": pct(ts, 0.99)}
        out[mode] = res
        del ls
    broker.destroy()
    print(json.dumps({"rccl_rtt": out, "loader_batches": loader_batches[0]}))


if __name__ == "__main__":
    main()
