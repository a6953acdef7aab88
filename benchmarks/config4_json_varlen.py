#!/usr/bin/env python3
"""BASELINE config 4: variable-length JSON records, on-device pad/stack -> bf16 (HIP collate), batch 256.

Records are JSON arrays of 16..256 numbers ("[-12.34, 5.06, ...]", ~1 KiB of text on
average), as in the reference README's ``json.loads(record.value)`` example.  By default
(decode='device') the workers only walk the record headers (the stage kernel counts each row's
elements and checks it is "simple"; --json-count host: the workers pre-scan each text in place),
and the gfx950 kernel (json_span.hip) reads the texts straight from the pinned broker logs,
verifies the RecordBatch CRCs, parses, pads, stacks and casts.  --decode host: the workers
frame + copy the text into the ring (json_parse.hip parses it); --json-parse host: the
workers parse every number.  The reference cannot collate this at all (variable-length lists
fail default_collate).

Usage: python benchmarks/config4_json_varlen.py [--steps K] [--device cuda:0]
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch-size", type=int, default=256)
    # config 2's worker count; the result line records it (round 2 quoted an 8-worker run as 4)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--min-len", type=int, default=16)
    ap.add_argument("--max-len", type=int, default=256)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--json-parse", default="auto", choices=["auto", "device", "host"])
    ap.add_argument("--h2d", default="auto", choices=["auto", "dma", "zerocopy"])
    ap.add_argument("--decode", default="auto", choices=["auto", "device", "host"])
    ap.add_argument("--json-count", default="auto", choices=["auto", "device", "host"],
                    help="who counts the elements of device-parsed rows: the stage kernel, or the workers")
    ap.add_argument("--slots-per-worker", type=int, default=None)
    ap.add_argument("--event-every", type=int, default=None)
    ap.add_argument("--prefetch", type=int, default=2)
    ap.add_argument("--verify", default="deliver", choices=["deliver", "commit"])
    ap.add_argument("--coalesce", type=int, default=None, help="batches per launch (default: the loader's)")
    ap.add_argument("--pad-to", type=int, default=None,
                    help="a fixed width (e.g. --max-len): the parse kernel counts each row itself "
                         "(no json_count_kernel); default: the batch's longest row, rounded up to pad_multiple")
    ap.add_argument("--lockstep", default="off", choices=["off", "rccl"],
                    help="rccl: the per-step RCCL agreement at world 1 (a one-rank nccl group), as under DDP")
    return ap.parse_args(argv)


def run(args, sync=None) -> dict:
    """One config-4 measurement; ``sync`` (optional) is called before and after the timed steps
    (bench.py passes its barrier + synchronize)."""
    import torch

    from torchkafka_amd import DeviceLoader, JsonArray, KafkaDataset, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    class Json(KafkaDataset):
        schema = JsonArray()

    url = f"shm://tkcfg4-{os.getpid()}"
    b = SyntheticBroker.create(url, log_capacity=1 << 33)
    try:
        b.create_topic("json", args.partitions)
        B = args.batch_size
        per_part = int(math.ceil((args.steps + args.warmup + 8 * args.workers) * B * 1.3 / args.partitions))
        t = time.perf_counter()
        b.fill("json", per_part, "json_f32", size=args.min_len, max_size=args.max_len, threads=args.partitions)
        fill_s = time.perf_counter() - t
        own_group = False
        if args.lockstep == "rccl" and not torch.distributed.is_initialized():
            import socket

            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            torch.distributed.init_process_group("nccl", rank=0, world_size=1)
            torch.distributed.all_reduce(torch.ones(1, device=args.device))  # torch's communicator, as DDP
            own_group = True
        dl = DeviceLoader(Json.placeholder(), B, num_workers=args.workers, device=args.device, dtype=torch.bfloat16,
                          json_parse=args.json_parse, h2d=args.h2d, decode=args.decode, json_count=args.json_count,
                          slots_per_worker=args.slots_per_worker, event_every=args.event_every, prefetch=args.prefetch,
                          verify=args.verify, lockstep="rccl" if args.lockstep == "rccl" else True,
                          **({"coalesce": args.coalesce} if args.coalesce else {}),
                          **({"pad_to": args.pad_to} if args.pad_to else {}),
                          worker_init_fn=Json.init_worker("json", bootstrap_servers=url, group_id="cfg4",
                                                          auto_offset_reset="earliest"))
        it = iter(auto_commit(dl))
        for _ in range(args.warmup):
            x, lens = next(it)
        mirror_on = bool(getattr(dl._run, "mirror", False))
        transport = dict(dl.lockstep_info).get("transport")
        if x.is_cuda:
            torch.cuda.synchronize()
        if sync is not None:
            sync()
        dl.reset_stats()
        t0 = time.perf_counter()
        rows = 0
        for _ in range(args.steps):
            x, lens = next(it)
            rows += x.shape[0]
        if x.is_cuda:
            torch.cuda.synchronize()
        if sync is not None:
            sync()
        el = time.perf_counter() - t0
        st = dl.stats_summary()
        it.close()
        dl.close()
        if own_group:
            torch.distributed.destroy_process_group()
        text_bytes = b.partition_stats("json", 0)["log_bytes"] / max(1, b.end_offset("json", 0))
        return {"config": 4, "metric": "JSON records/s to GPU (bf16 padded), per-batch commit",
                "value": round(rows / el), "ms_per_step": round(el / args.steps * 1e3, 4),
                "gb_per_s_text": round(rows / el * text_bytes / 1e9, 2),
                "batch_size": B, "workers": args.workers, "partitions": args.partitions,
                "json_parse": args.json_parse, "h2d": args.h2d, "verify": dl.verify,
                "lockstep": transport,
                "decode": (("device (json_span.hip from an HBM mirror filled by SDMA copies)"
                            if mirror_on else "device (json_span.hip from the pinned logs)")
                           if dl.plan.json_span else args.decode),
                "json_count": "device" if dl.plan.json_count else "workers",
                "pad_to": args.pad_to,
                "timed_s": round(el, 4), "steps": args.steps,
                "avg_record_bytes": round(text_bytes),
                "last_batch_shape": list(x.shape),
                "commits": st["commits"], "commit_latency_p50_us": round(st["commit_latency_p50_us"], 2),
                "commit_latency_p99_us": round(st["commit_latency_p99_us"], 2),
                "device": args.device, "fill_s": round(fill_s, 2), "loader": st}
    finally:
        b.destroy()


def main():
    print(json.dumps(run(parse())))


if __name__ == "__main__":
    main()
