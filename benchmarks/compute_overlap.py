#!/usr/bin/env python3
"""What the loader costs a co-running training job: a bf16 GEMM stream beside the loader.

The reference keeps batches on the CPU (kafka_dataset.py:156-162 plus the DataLoader's collate,
SURVEY E5), so its data path takes nothing from the GPU.  This framework decodes on the GPU, so
its decode kernels share CUs, LDS and the memory system with the model they feed.  This block
measures that share directly:

  1. ``gemm_alone``: ``--gemms`` back-to-back ``torch.matmul`` of two bf16 [G, G] matrices
     (MFMA-bound; G = 8192 by default, 1.1 TFLOP each) on the user's stream, each bracketed by
     HIP events -> TFLOP/s;
  2. ``loader_alone``: ``--steps`` steps of the loader (config 2's fixed-width f32[256] -> bf16,
     or config 4's JSON -> bf16) -> records/s;
  3. ``together``: the same loader for ``--steps`` steps while the user's stream is kept
     ``--depth`` GEMMs deep (a new GEMM is queued whenever the oldest completed; checked every
     ``--poll`` steps) -> the loader's records/s and the GEMMs' TFLOP/s beside it.

A GEMM's TFLOP/s is FLOPs over its own event-timed execution (``sum``: the busy time of the
GEMMs that ran inside the window), so a host that queued late cannot flatter or hurt it; the
``span`` rate (first start to last end) is reported next to it with ``dry_gaps_ms``, the time
the stream ran without a queued GEMM.  ``gemm_slowdown_pct`` = how much longer the stream takes
per GEMM beside the loader (span-based: a host that stopped feeding the stream counts), with
``dry_gaps_ms`` beside it; ``gemm_kernel_slowdown_pct`` = the per-GEMM kernel time alone (p50).
The loader's window ends when its last step returned (with ``verify="deliver"`` that is after the
last batch's device verdict).

Usage: python benchmarks/compute_overlap.py [--workload config2|config4] [--h2d auto|zerocopy|dma]
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
    ap.add_argument("--workload", default="config2", choices=["config2", "config4"])
    ap.add_argument("--steps", type=int, default=30000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--gemm", type=int, default=8192, help="M = N = K of the bf16 GEMM")
    ap.add_argument("--gemms", type=int, default=60, help="GEMMs of the alone measurement")
    ap.add_argument("--depth", type=int, default=3, help="GEMMs kept queued on the user's stream")
    ap.add_argument("--poll", type=int, default=8, help="loader steps between checks of the GEMM queue")
    ap.add_argument("--h2d", default="auto", choices=["auto", "dma", "zerocopy"])
    ap.add_argument("--verify", default="deliver", choices=["deliver", "commit"])
    ap.add_argument("--device", default="cuda:0")
    return ap.parse_args(argv)


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(len(xs) * q))] if xs else 0.0


class GemmStream:
    """bf16 GEMMs queued on the current stream, each between two timing events."""

    def __init__(self, torch, n: int, device):
        self.torch = torch
        g = torch.Generator(device=device).manual_seed(0)
        self.a = torch.randn((n, n), device=device, dtype=torch.bfloat16, generator=g)
        self.b = torch.randn((n, n), device=device, dtype=torch.bfloat16, generator=g)
        self.c = torch.empty((n, n), device=device, dtype=torch.bfloat16)
        self.flops = 2.0 * n * n * n
        self.pending = []  # (start, end) events, oldest first
        self.done = []

    def push(self) -> None:
        cuda = self.torch.cuda
        s, e = cuda.Event(enable_timing=True), cuda.Event(enable_timing=True)
        s.record()
        self.torch.matmul(self.a, self.b, out=self.c)
        e.record()
        self.pending.append((s, e))

    def refill(self, depth: int) -> None:
        while self.pending and self.pending[0][1].query():
            self.done.append(self.pending.pop(0))
        while len(self.pending) < depth:
            self.push()

    def drain(self) -> None:
        self.torch.cuda.synchronize()
        self.done.extend(self.pending)
        self.pending = []

    def report(self, cut_ms: float | None = None) -> dict:
        """Per-GEMM execution times (ms) of the finished GEMMs; ``cut_ms``: only GEMMs that started
        before that many ms after the first one (the loader's window)."""
        if not self.done:
            return {}
        t0 = self.done[0][0]
        runs = []
        for s, e in self.done:
            st = t0.elapsed_time(s)
            if cut_ms is not None and st > cut_ms:
                break
            runs.append((st, t0.elapsed_time(e)))
        ms = [b - a for a, b in runs]
        gaps = sum(max(0.0, runs[i + 1][0] - runs[i][1]) for i in range(len(runs) - 1))
        span = runs[-1][1] - runs[0][0]
        return {"gemms": len(runs), "ms_per_gemm_p50": round(_pct(ms, 0.5), 4),
                "ms_per_gemm_max": round(max(ms), 4),
                "tflops_sum": round(len(runs) * self.flops / (sum(ms) * 1e-3) / 1e12, 1),
                "tflops_span": round(len(runs) * self.flops / (span * 1e-3) / 1e12, 1),
                "dry_gaps_ms": round(gaps, 3)}


def run(args, sync=None) -> dict:
    import torch

    from torchkafka_amd import DeviceLoader, FixedWidth, JsonArray, KafkaDataset, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    sync = sync or (lambda: torch.cuda.synchronize())
    dev = torch.device(args.device)

    class Records(KafkaDataset):
        schema = FixedWidth(torch.float32, (args.dim,))

    class Json(KafkaDataset):
        schema = JsonArray()

    cfg4 = args.workload == "config4"
    ds = Json if cfg4 else Records
    url = f"shm://tkcompute-{os.getpid()}"
    B = args.batch_size
    b = SyntheticBroker.create(url, log_capacity=1 << 34, index_capacity=1 << 22)
    try:
        b.create_topic("t", args.partitions)
        per_part = int(math.ceil((2 * args.steps + args.warmup + 16 * args.workers) * B * 1.3 / args.partitions))
        t = time.perf_counter()
        if cfg4:
            b.fill("t", per_part, "json_f32", size=16, max_size=256, threads=args.partitions)
        else:
            b.fill("t", per_part, "fixed_f32", size=args.dim, threads=args.partitions, keyed=True)
        fill_s = time.perf_counter() - t
        dl = DeviceLoader(ds.placeholder(), B, num_workers=args.workers, device=dev, dtype=torch.bfloat16,
                          h2d=args.h2d, verify=args.verify,
                          worker_init_fn=ds.init_worker("t", bootstrap_servers=url, group_id="compute",
                                                        auto_offset_reset="earliest"))
        it = iter(auto_commit(dl))
        torch.cuda.set_device(dev)
        gs = GemmStream(torch, args.gemm, dev)

        def first(x):
            return x[0] if isinstance(x, (tuple, list)) else x

        for _ in range(args.warmup):
            next(it)
        for _ in range(4):  # hipBLASLt's kernel choice and workspace
            gs.push()
        gs.drain()
        gs.done = []

        # 1. GEMMs alone
        sync()
        for _ in range(args.gemms):
            gs.push()
        gs.drain()
        alone = gs.report()
        gs.done = []

        # 2. the loader alone
        dl.reset_stats()
        sync()
        t0 = time.perf_counter()
        rows = 0
        for _ in range(args.steps):
            rows += first(next(it)).shape[0]
        el_alone = time.perf_counter() - t0
        sync()

        # 3. together: the stream is kept `depth` GEMMs deep from before t0 to the loader's last step
        dl.reset_stats()
        sync()
        gs.refill(args.depth)
        t0 = time.perf_counter()
        rows2 = 0
        for k in range(args.steps):
            rows2 += first(next(it)).shape[0]
            if k % args.poll == 0:
                gs.refill(args.depth)
        el_both = time.perf_counter() - t0
        cut_ms = el_both * 1e3
        gs.drain()
        beside = gs.report(cut_ms)
        st = dl.stats_summary()
        decode = (("device, HBM mirror filled by SDMA copies" if dl.plan.mirror
                   else "device, zero-copy from the pinned logs")
                  if (dl.plan.span or getattr(dl.plan, "json_span", False)) else "host workers")
        it.close()
        dl.close()
        out = {
            "workload": ("config 4: JSON arrays -> bf16" if cfg4 else
                         f"config 2: FixedWidth f32[{args.dim}] -> bf16"),
            "h2d": args.h2d, "decode": decode, "verify": args.verify,
            "gemm": f"torch.matmul bf16 [{args.gemm}, {args.gemm}] x [{args.gemm}, {args.gemm}] on the user stream",
            "gemm_alone": alone,
            "loader_alone_records_per_s": round(rows / el_alone, 1),
            "together": {"records_per_s": round(rows2 / el_both, 1), "timed_s": round(el_both, 4),
                         "steps": args.steps, "gemm": beside, "depth": args.depth,
                         "commits": st["commits"]},
            "fill_s": round(fill_s, 2),
        }
        if alone and beside:
            # what the training job sees: its stream's span per GEMM (kernel time AND the gaps when
            # the host, blocked in next(), stopped feeding it) against alone
            out["gemm_slowdown_pct"] = round((alone["tflops_span"] / beside["tflops_span"] - 1) * 100, 2)
            out["dry_gaps_ms"] = beside["dry_gaps_ms"]
            out["gemm_kernel_slowdown_pct"] = round(
                (beside["ms_per_gemm_p50"] / alone["ms_per_gemm_p50"] - 1) * 100, 2)
            out["gemm_tflops_ratio"] = round(beside["tflops_sum"] / alone["tflops_sum"], 4)
            out["loader_ratio"] = round(out["together"]["records_per_s"] / out["loader_alone_records_per_s"], 4)
        return out
    finally:
        b.destroy()


def main():
    print(json.dumps(run(parse())))


if __name__ == "__main__":
    main()
