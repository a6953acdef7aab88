#!/usr/bin/env python3
"""Headline benchmark: Kafka records/sec delivered to the GPU with a commit after every batch.

BASELINE.json metric "Kafka records/sec to GPU with per-batch commit, at
1/2/4/8 MI355X".  Configurations (BASELINE.json ``configs``):

  * N = 1 : config 2 -- 1x MI355X, num_workers=4, 8-partition topic,
            fixed-width float32 records (256 x f32 = 1 KiB), pinned ring +
            hipMemcpyAsync on a side stream, gfx950 collate kernel -> bf16;
  * N > 1 : config 3 -- one process per GPU (torchrun), 8 partitions per rank
            (64 at N = 8), static rank sharding, auto_commit lock-stepped by an
            RCCL all-reduce over xGMI every step.

A step = one batch of ``--batch-size`` records per rank consumed from the
synthetic broker, packed in pinned memory, copied to the GPU, collated to
bf16 by the HIP kernel, handed to the user, and its offsets committed (the
commit of batch k happens when batch k+1 is requested, as in the reference's
auto_commit).  Records are synthetic Kafka RecordBatch v2 records produced
into the shared-memory broker before timing (a retained backlog).
Weak scaling: per-rank work is fixed as N grows.

Usage: python bench.py [--gpus N --steps K --warmup W]
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

BASELINE_METRIC = "Kafka records/sec to GPU with per-batch commit, at 1/2/4/8 MI355X"
# reference measured on config 2's shape without a GPU (bs=256, 1 KiB f32[256], nw=4)
BASELINE_VALUE = 337237.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--dim", type=int, default=256, help="float32 elements per record")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--partitions-per-gpu", type=int, default=8)
    ap.add_argument("--slots-per-worker", type=int, default=None, help="ring depth (default: loader's auto)")
    ap.add_argument("--prefetch", type=int, default=2)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "f16", "f32"])
    ap.add_argument("--records-per-batch", type=int, default=64, help="Kafka RecordBatch size in the log")
    ap.add_argument("--no-crc", action="store_true", help="skip CRC32C verification (kafka-python check_crcs)")
    ap.add_argument("--device", default=None, help="override device (e.g. cpu for a dry run)")
    ap.add_argument("--stats", action="store_true", help="print loader stats to stderr")
    ap.add_argument("--in-order", action="store_true", help="strict worker round-robin delivery")
    ap.add_argument("--event-every", type=int, default=None)
    ap.add_argument("--h2d", default="auto", choices=["auto", "dma", "zerocopy", "direct"])
    ap.add_argument("--copy-streams", type=int, default=4)
    ap.add_argument("--mirror-chunk-mib", type=int, default=8,
                    help="--h2d dma with device decode: MiB per hipMemcpyAsync into the HBM log mirror")
    ap.add_argument("--mirror-chunks", type=int, default=None, help="--h2d dma: HBM mirror buffers per partition")
    ap.add_argument("--lockstep-depth", type=int, default=2)
    ap.add_argument("--coalesce", type=int, default=8, help="staged batches collated per kernel launch")
    ap.add_argument("--coalesce-wait-us", type=int, default=50, help="adaptive coalescing wait while the GPU is busy")
    ap.add_argument("--no-numa", action="store_true", help="do not bind ranks to their GPU's NUMA node")
    ap.add_argument("--decode", default="auto", choices=["auto", "device", "host"],
                    help="device: gfx950 RecordBatch decode + CRC from the pinned logs; host: workers CRC-check + pack")
    ap.add_argument("--lockstep", default="auto", choices=["auto", "off", "rccl", "host"],
                    help="cross-rank step/commit agreement: auto = RCCL at N > 1, none at N = 1; rccl/host force "
                         "it (also at N = 1) over the native RCCL communicator / the process group's all-reduce")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 with a gloo group (rehearse N > 1 ranks on a one-GPU box)")
    ap.add_argument("--steady-steps", type=int, default=None,
                    help="steps of the steady-state block timed after the headline (default: max(50 x ring "
                         "slots, 4000); 0 skips it)")
    return ap.parse_args()


def main() -> int:
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        print(f"[bench] warning: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
    from torchkafka_amd.broker import SyntheticBroker
    from torchkafka_amd.parallel import shard_partitions
    from torchkafka_amd.utils.topology import bind_to_gpu_numa

    if not args.device and not args.no_numa:
        # the broker log this rank fills, its ring and its workers all live on its GPU's socket
        bind_to_gpu_numa(local_rank)

    dtype = {"bf16": torch.bfloat16, "fp8": torch.float8_e4m3fn, "f16": torch.float16, "f32": torch.float32}[args.dtype]
    device = torch.device(args.device) if args.device else torch.device("cuda", 0 if args.same_device else local_rank)
    # lockstep: the agreement every step runs before a batch is delivered and committed
    if args.lockstep == "off":
        lockstep = False
    elif args.lockstep == "auto":
        lockstep = "host" if args.same_device else True
    elif world == 1:
        lockstep = "always"  # agree every step even alone: RCCL on an nccl group, all-reduce on gloo
    else:
        lockstep = args.lockstep

    class Records(KafkaDataset):
        schema = FixedWidth(torch.float32, (args.dim,))

    # --- broker: one per job (all ranks of a torchrun share the agent's pid and port)
    tag = f"{os.getppid()}-{os.environ.get('MASTER_PORT', '0')}" if world > 1 else f"{os.getpid()}"
    url = f"shm://tkbench-{tag}"
    n_parts = args.partitions_per_gpu * world
    B = args.batch_size
    broker = SyntheticBroker.create(url, log_capacity=1 << 34, index_capacity=1 << 22)
    broker.create_topic("bench", n_parts)
    # backlog per owned partition: every batch the timed loop and the warm-up consume, plus what the
    # workers prefetch into their ring slots, with headroom
    mine = shard_partitions(n_parts, rank, world)
    ring_guess = args.workers * (args.slots_per_worker or 8)
    steady = args.steady_steps if args.steady_steps is not None else max(50 * ring_guess, 4000)
    batches = args.warmup + args.steps + steady + args.workers * ((args.slots_per_worker or 8) + 2)
    per_part = int(math.ceil(batches * B * 1.25 / max(1, len(mine)))) + B
    t_fill = time.perf_counter()
    broker.fill("bench", per_part, "fixed_f32", size=args.dim, partitions=mine,
                records_per_batch=args.records_per_batch, threads=min(16, len(mine)))
    t_fill = time.perf_counter() - t_fill

    use_gloo = device.type != "cuda" or args.same_device or args.lockstep == "host"
    if world > 1 or args.lockstep in ("rccl", "host"):
        # no CUDA touched yet: the loader forks its workers before HIP is initialised
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        dist.init_process_group("gloo" if use_gloo else "nccl", rank=rank, world_size=world)

    loader = DeviceLoader(
        Records.placeholder(), B, num_workers=args.workers, device=device, dtype=dtype,
        slots_per_worker=args.slots_per_worker, prefetch=args.prefetch, rank=rank, world_size=world,
        in_order=args.in_order, h2d=args.h2d, copy_streams=args.copy_streams, lockstep_depth=args.lockstep_depth,
        event_every=args.event_every, numa_bind=not args.no_numa, coalesce=args.coalesce,
        coalesce_wait_us=args.coalesce_wait_us, decode=args.decode, lockstep=lockstep,
        mirror_chunk_mib=args.mirror_chunk_mib,
        **({"mirror_chunks": args.mirror_chunks} if args.mirror_chunks else {}),
        worker_init_fn=Records.init_worker("bench", bootstrap_servers=url, group_id="bench",
                                           auto_offset_reset="earliest", check_crcs=not args.no_crc),
    )
    it = iter(auto_commit(loader))
    x = next(it)  # forks workers, initialises HIP/RCCL
    if device.type == "cuda":
        torch.cuda.set_device(device)

    def barrier():
        dist.barrier(device_ids=[local_rank] if device.type == "cuda" and not use_gloo else None)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if world > 1:
            barrier()
            if device.type == "cuda":
                torch.cuda.synchronize(device)

    for _ in range(max(0, args.warmup - 1)):
        x = next(it)
    sync()
    loader.reset_stats()
    # what the workers filled ahead of the consumer: a short timed region may only drain these
    occ = loader.ring_occupancy()
    t0 = time.perf_counter()
    rows = 0
    for _ in range(args.steps):
        x = next(it)
        rows += x.shape[0]
    sync()
    elapsed = time.perf_counter() - t0
    stats = loader.stats_summary()

    def job_rate(el: float, nrows: int) -> tuple[float, float]:
        """whole-job aggregate: records of every rank over the slowest rank's time"""
        if world == 1:
            return el, float(nrows)
        t = torch.tensor([el, float(nrows)], dtype=torch.float64, device="cpu" if use_gloo else device)
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        return float(tmax[0]), float(t[1])

    elapsed, total_rows = job_rate(elapsed, rows)
    value = total_rows / elapsed

    # Steady state, same process, right after the headline: many times the ring depth, so the
    # batches the workers had prefilled before t0 are a small part of it and the producer side
    # (fetch, pack, publish) is inside the timed region.
    steady_out = None
    if steady > 0:
        n_slots = occ["n_slots"] or ring_guess
        s_steps = steady
        loader.reset_stats()
        sync()
        occ_s = loader.ring_occupancy()
        if args.stats:
            print(json.dumps({"ring_at_steady_t0": occ_s}), file=sys.stderr)
        t1 = time.perf_counter()
        srows = 0
        for _ in range(s_steps):
            x = next(it)
            srows += x.shape[0]
        sync()
        s_el, s_total = job_rate(time.perf_counter() - t1, srows)
        s_stats = loader.stats_summary()
        steady_out = {
            "steps": s_steps,
            "timed_s": round(s_el, 6),
            "records_per_s": round(s_total / s_el, 1),
            "ms_per_step": round(s_el / s_steps * 1000, 4),
            "gb_per_s": round(s_total / s_el * args.dim * 4 / 1e9, 3),
            "ring_slots": n_slots,
            "prefilled_slots_at_t0": occ_s["prefilled"],
            "steps_per_ring": round(s_steps / max(1, n_slots), 1),
            "vs_baseline": round(s_total / s_el / BASELINE_VALUE, 3),
            "commit_p50_us": round(s_stats["commit_p50_us"], 2),
            "commit_p99_us": round(s_stats["commit_p99_us"], 2),
            "commit_latency_p50_us": round(s_stats["commit_latency_p50_us"], 2),
            "commit_latency_p99_us": round(s_stats["commit_latency_p99_us"], 2),
            "worker_fill_us_per_batch": round(s_stats.get("worker_fill_us_per_batch", 0.0), 2),
        }

    # check what landed on the device: the last batch's records must be this rank's partitions
    xf = x.float()
    parts = set(int(p) for p in xf[:, 1].tolist())
    assert parts <= set(mine), f"rank {rank} received foreign partitions {parts - set(mine)}"

    it.close()  # normal end of the auto_commit generator: final commit + worker shutdown
    if world > 1:
        barrier()
    committed = broker.committed_offsets("bench", "bench")
    if rank == 0:
        if args.stats:
            print(json.dumps({"loader_stats": stats, "fill_s": t_fill,
                              "committed_sample": dict(list(committed.items())[:4])}),
                  file=sys.stderr)
        out = {
            "metric": BASELINE_METRIC,
            "value": round(value, 1),
            "unit": "records/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_VALUE, 3),
            "dtype": args.dtype,
            "data": ("synthetic (Kafka RecordBatch v2 records in the shared-memory broker, "
                     "random-free deterministic f32)"),
            "config": {
                "model": (f"KafkaDataset FixedWidth f32[{args.dim}] ({args.dim * 4} B records) -> {args.dtype} "
                          "via gfx950 collate"),
                "global_batch": B * world,
                "seq_len": args.dim,
                "parallelism": f"dp{world}",
                "partitions": n_parts,
                "num_workers": args.workers,
                "commit": "auto_commit per batch" + (
                    "" if not lockstep or (lockstep is True and world == 1)
                    else ", lockstep (gloo all-reduce)" if use_gloo else ", RCCL lockstep"),
                "h2d": loader._resolve_h2d(loader._slot_capacity()) if device.type == "cuda" else "n/a (cpu)",
                "decode": ("host workers" if not loader._span() else
                           "device (gfx950 CRC32C + decode from an HBM mirror filled by SDMA copies)"
                           if loader._mirror() else "device (gfx950 CRC32C + decode from pinned logs)"),
                "bytes_per_step_per_gpu": B * args.dim * 4,
                "gb_per_s": round(value * args.dim * 4 / 1e9, 3),
                "commit_p99_us": round(stats["commit_p99_us"], 2),
            },
            # request of batch k+1 -> batch k's offsets stored, incl. the lockstep agreement and the
            # wait for batch k's on-device CRC verdict (steady-state block when it ran)
            "commit_latency_p50_us": round((s_stats if steady_out else stats)["commit_latency_p50_us"], 2),
            "commit_latency_p99_us": round((s_stats if steady_out else stats)["commit_latency_p99_us"], 2),
            "timed_region_s": round(elapsed, 6),
            "prefilled_slots_at_t0": occ["prefilled"],
            "ring_slots": occ["n_slots"],
            "steady_state": steady_out,
        }
        print(json.dumps(out))
    loader.close()
    if world > 1:
        barrier()
        dist.destroy_process_group()
    if rank == 0:
        broker.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
