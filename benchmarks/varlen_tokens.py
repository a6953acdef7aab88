#!/usr/bin/env python3
"""Variable-length int32 token-id records -> padded int64 batch on the GPU, commit after every batch.

Not a BASELINE config: the language-model shape of BASELINE config 4 (variable-length records,
on-device pad/stack, batch 256), with raw little-endian int32 token ids instead of JSON text --
what a pre-tokenised training stream looks like.  Records hold 64..512 tokens (~1.1 KiB on
average).  ``--decode device`` (default): the workers only walk the record headers and the gfx950
varlen_span_kernel reads the values straight from the pinned broker logs (CRC32C verified on the
device); ``--decode host``: the workers CRC-check and pack CSR into the ring, the varlen collate
kernel pads.

Usage: python benchmarks/varlen_tokens.py [--steps K] [--decode device|host]
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--min-len", type=int, default=64)
    ap.add_argument("--max-len", type=int, default=512)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--decode", default="auto", choices=["auto", "device", "host"])
    ap.add_argument("--h2d", default="auto", choices=["auto", "dma", "zerocopy"])
    ap.add_argument("--coalesce", type=int, default=None, help="batches per launch (default: the loader's)")
    ap.add_argument("--lockstep", default="off", choices=["off", "rccl"],
                    help="rccl: the per-step RCCL agreement at world 1 (a one-rank nccl group), as under DDP")
    args = ap.parse_args()

    import torch

    from torchkafka_amd import DeviceLoader, KafkaDataset, VarLen, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    class Tokens(KafkaDataset):
        schema = VarLen(torch.int32)

    url = f"shm://tktok-{os.getpid()}"
    b = SyntheticBroker.create(url, log_capacity=1 << 33)
    try:
        b.create_topic("tok", args.partitions)
        B = args.batch_size
        per_part = int(math.ceil((args.steps + args.warmup + 16 * args.workers) * B * 1.3 / args.partitions))
        t = time.perf_counter()
        b.fill("tok", per_part, "tokens_i32", size=args.min_len, max_size=args.max_len, threads=args.partitions)
        fill_s = time.perf_counter() - t
        if args.lockstep == "rccl":
            import socket

            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            torch.distributed.init_process_group("nccl", rank=0, world_size=1)
            torch.distributed.all_reduce(torch.ones(1, device=args.device))  # torch's communicator, as DDP
        dl = DeviceLoader(Tokens.placeholder(), B, num_workers=args.workers, device=args.device, dtype=torch.int64,
                          decode=args.decode, h2d=args.h2d, lockstep="rccl" if args.lockstep == "rccl" else True,
                          **({"coalesce": args.coalesce} if args.coalesce else {}),
                          worker_init_fn=Tokens.init_worker("tok", bootstrap_servers=url, group_id="tok",
                                                            auto_offset_reset="earliest"))
        it = iter(auto_commit(dl))
        for _ in range(args.warmup):
            x, lens = next(it)
        mirror_on = bool(getattr(dl._run, "mirror", False))
        transport = dict(dl.lockstep_info).get("transport")
        torch.cuda.synchronize()
        dl.reset_stats()
        t0 = time.perf_counter()
        rows = 0
        for _ in range(args.steps):
            x, lens = next(it)
            rows += x.shape[0]
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        st = dl.stats_summary()
        decode = (("device (varlen_span_kernel from an HBM mirror filled by SDMA copies)" if mirror_on
                   else "device (varlen_span_kernel from the pinned logs)") if dl.plan.var_span else "host workers")
        it.close()
        dl.close()
        if args.lockstep == "rccl":
            torch.distributed.destroy_process_group()
        rec_bytes = b.partition_stats("tok", 0)["log_bytes"] / max(1, b.end_offset("tok", 0))
        print(json.dumps({"metric": "int32 token records/s to GPU (int64 padded), per-batch commit",
                          "value": round(rows / el), "ms_per_step": round(el / args.steps * 1e3, 4),
                          "timed_s": round(el, 4), "steps": args.steps, "batch_size": B, "workers": args.workers,
                          "decode": decode, "h2d": args.h2d, "lockstep": transport,
                          "avg_record_bytes": round(rec_bytes),
                          "gb_per_s": round(rows / el * rec_bytes / 1e9, 2), "last_batch_shape": list(x.shape),
                          "fill_s": round(fill_s, 2), "loader": st}))
    finally:
        b.destroy()


if __name__ == "__main__":
    main()
