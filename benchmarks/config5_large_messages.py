#!/usr/bin/env python3
"""BASELINE config 5 (stress): 1 MiB messages, 128 partitions, pinned ring, p99 commit latency.

Each record is 262,144 float32 (1 MiB); batches of ``--batch-size`` records are described by
the workers in pinned ring slots (``slots_per_worker`` deep: 2 = double-buffered) and decoded
on the device straight from the pinned logs (CRC32C + cast to bf16, span_decode.hip), then
committed after use.  Reports records/s, GB/s and the commit latency distribution (p50/p99) measured
around every commit.  Reference yardstick: 3,481 records/s (3.40 GiB/s)
at batch 8 with 4 workers, CPU only.

Usage: python benchmarks/config5_large_messages.py [--steps K] [--device cuda:0]
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

YARDSTICK = 3481.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=8)
    # Device decode leaves the workers only the record headers (~25-33 us per 8 MiB batch), so the ring
    # depth sets the commit latency (Little's law: in-flight bytes / link rate): 2 workers x 2 slots
    # 51.3 k rec/s, latency p99 0.78 ms; 4 workers 45.4 k, 1.6 ms; 8 workers 45.8 k, 3.0 ms
    # (profiles/r02_s3_final/config5_w*.log)
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--partitions", type=int, default=128)
    ap.add_argument("--slots-per-worker", type=int, default=2)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--h2d", default="auto", choices=["auto", "dma", "zerocopy", "direct"])
    ap.add_argument("--verify", default="deliver", choices=["deliver", "commit"])
    return ap.parse_args(argv)


def run(args, sync=None) -> dict:
    """One config-5 measurement; ``sync`` (optional) brackets the timed steps (bench.py's barrier)."""
    import torch

    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    D = 1 << 18  # floats per record = 1 MiB

    class Big(KafkaDataset):
        schema = FixedWidth(torch.float32, (D,))

    url = f"shm://tkcfg5-{os.getpid()}"
    B = args.batch_size
    total = (args.steps + args.warmup + args.workers * (args.slots_per_worker + 2)) * B
    per_part = int(math.ceil(total * 1.1 / args.partitions))
    b = SyntheticBroker.create(url, log_capacity=(per_part + 4) * (D * 4 + 64), index_capacity=per_part + 16)
    try:
        b.create_topic("big", args.partitions)
        t = time.perf_counter()
        b.fill("big", per_part, "fixed_f32", size=D, records_per_batch=1, threads=min(16, args.partitions))
        fill_s = time.perf_counter() - t
        dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
        dl = DeviceLoader(Big.placeholder(), B, num_workers=args.workers, device=args.device, dtype=dtype,
                          slots_per_worker=args.slots_per_worker, prefetch=1, h2d=args.h2d, verify=args.verify,
                          worker_init_fn=Big.init_worker("big", bootstrap_servers=url, group_id="cfg5",
                                                         auto_offset_reset="earliest"))
        it = iter(auto_commit(dl))
        for _ in range(args.warmup):
            x = next(it)
        if x.is_cuda:
            torch.cuda.synchronize()
        if sync is not None:
            sync()
        dl.reset_stats()
        t0 = time.perf_counter()
        rows = 0
        for _ in range(args.steps):
            x = next(it)
            rows += x.shape[0]
        if x.is_cuda:
            torch.cuda.synchronize()
        if sync is not None:
            sync()
        el = time.perf_counter() - t0
        st = dl.stats_summary()
        it.close()
        dl.close()
        v = rows / el
        return {"config": 5, "metric": "1 MiB records/s to GPU, per-batch commit", "value": round(v, 1),
                "gb_per_s": round(v * D * 4 / 1e9, 2), "vs_yardstick": round(v / YARDSTICK, 2),
                "steps": args.steps, "timed_s": round(el, 4), "commits": st["commits"],
                "commit_p50_us": round(st["commit_p50_us"], 2), "commit_p99_us": round(st["commit_p99_us"], 2),
                "commit_latency_means": "request of batch k+1 -> batch k's offsets stored (incl. its CRC verdict)",
                "commit_latency_p50_us": round(st["commit_latency_p50_us"], 2),
                "commit_latency_p99_us": round(st["commit_latency_p99_us"], 2),
                "batch_size": B, "partitions": args.partitions, "workers": args.workers,
                "slots_per_worker": args.slots_per_worker, "verify": dl.verify, "device": args.device,
                "fill_s": round(fill_s, 1), "loader": st}
    finally:
        b.destroy()


def main():
    print(json.dumps(run(parse())))


if __name__ == "__main__":
    main()
