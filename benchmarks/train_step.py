#!/usr/bin/env python3
"""The loader inside a real training step: does feeding a model from Kafka cost the model anything?

The reference's data path takes nothing from the GPU: batches stay CPU tensors
(/root/reference/src/kafka_dataset.py:156-162, collate on the CPU).  This framework decodes on the
GPU, so its kernels share the CUs with the model they feed.  This block runs the same bf16 MLP
training step two ways, alternated (A B A B) so drift on the box hits both:

  * ``prestaged``: ``x`` cycles through 64 batches decoded once and kept on the device -- the step
    with a free data path;
  * ``loader``: ``for x in auto_commit(loader): loss = mlp(x); loss.backward(); opt.step()`` --
    every batch decoded on the GPU (config 2: FixedWidth f32[256] -> bf16; config 4: JSON arrays
    of 16..256 numbers -> bf16 padded to 256), verified, handed out and committed after the step.

``overhead_pct`` = loader step time over prestaged step time - 1 (median of the two pairs).  Both
loops are timed on the host between a synchronize before the first step and one after the last, so
any wait of ``next()`` on a decode (the CRC verdict with ``verify="deliver"``) is inside.

The model: Linear(256, H) -> GELU -> [Linear(H, H) -> GELU] x 2 -> Linear(H, 16), bf16, AdamW
(fused); H = 8192 by default, 1.21 ms per step at batch 256 on one MI355X (profiles/r06_s3).

Usage: python benchmarks/train_step.py [--workload config2|config4] [--h2d auto|zerocopy|dma]
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
    ap.add_argument("--steps", type=int, default=1500, help="timed steps per loop (each loop runs twice)")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--h2d", default="auto", choices=["auto", "dma", "zerocopy"])
    ap.add_argument("--verify", default="deliver", choices=["deliver", "commit"])
    ap.add_argument("--device", default="cuda:0")
    return ap.parse_args(argv)


def _model(torch, hidden: int, dev):
    nn = torch.nn
    m = nn.Sequential(nn.Linear(256, hidden), nn.GELU(), nn.Linear(hidden, hidden), nn.GELU(),
                      nn.Linear(hidden, hidden), nn.GELU(), nn.Linear(hidden, 16))
    m = m.to(device=dev, dtype=torch.bfloat16)
    try:
        opt = torch.optim.AdamW(m.parameters(), lr=1e-5, fused=True)
    except (RuntimeError, TypeError):
        opt = torch.optim.AdamW(m.parameters(), lr=1e-5, foreach=True)
    return m, opt


def run(args, sync=None) -> dict:
    import torch

    from torchkafka_amd import DeviceLoader, FixedWidth, JsonArray, KafkaDataset, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    sync = sync or (lambda: torch.cuda.synchronize())
    dev = torch.device(args.device)

    class Records(KafkaDataset):
        schema = FixedWidth(torch.float32, (256,))

    class Json(KafkaDataset):
        schema = JsonArray()

    cfg4 = args.workload == "config4"
    ds = Json if cfg4 else Records
    url = f"shm://tktrain-{os.getpid()}"
    B = args.batch_size
    b = SyntheticBroker.create(url, log_capacity=1 << 33, index_capacity=1 << 22)
    try:
        b.create_topic("t", args.partitions)
        per_part = int(math.ceil((2 * args.steps + 2 * args.warmup + 200 + 16 * args.workers) * B * 1.3
                                 / args.partitions))
        if cfg4:
            b.fill("t", per_part, "json_f32", size=16, max_size=256, threads=args.partitions)
        else:
            b.fill("t", per_part, "fixed_f32", size=256, threads=args.partitions, keyed=True)
        extra = {"pad_to": 256} if cfg4 else {}
        dl = DeviceLoader(ds.placeholder(), B, num_workers=args.workers, device=dev, dtype=torch.bfloat16,
                          h2d=args.h2d, verify=args.verify, **extra,
                          worker_init_fn=ds.init_worker("t", bootstrap_servers=url, group_id="train",
                                                        auto_offset_reset="earliest"))
        it = iter(auto_commit(dl))
        torch.cuda.set_device(dev)
        model, opt = _model(torch, args.hidden, dev)

        def step(x):
            if isinstance(x, (tuple, list)):  # var-len / JSON batches: (values, lengths)
                x = x[0]
            loss = model(x).float().pow(2).mean()
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)

        def first(x):
            return x[0] if isinstance(x, (tuple, list)) else x

        staged = [first(next(it)).clone() for _ in range(64)]
        for k in range(args.warmup):  # kernels chosen, optimiser state made, the loader warm
            step(staged[k % 64])
            next(it)
        sync()

        def prestaged():
            sync()
            t0 = time.perf_counter()
            for k in range(args.steps):
                step(staged[k % 64])
            sync()
            return (time.perf_counter() - t0) / args.steps * 1e3

        def from_loader():
            dl.reset_stats()
            sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step(next(it))
            sync()
            return (time.perf_counter() - t0) / args.steps * 1e3, dl.stats_summary()

        a1 = prestaged()
        b1, st1 = from_loader()
        a2 = prestaged()
        b2, st2 = from_loader()
        decode = (("device, HBM mirror filled by SDMA copies" if dl.plan.mirror
                   else "device, zero-copy from the pinned logs")
                  if (dl.plan.span or getattr(dl.plan, "json_span", False)) else "host workers")
        h2d = dl.plan.resolve_h2d(dl._slot_capacity())
        it.close()
        dl.close()
        ovh = sorted([(b1 / a1 - 1) * 100, (b2 / a2 - 1) * 100])
        flops = 6.0 * B * (256 * args.hidden + 2 * args.hidden * args.hidden + args.hidden * 16)
        return {
            "workload": ("config 4: JSON arrays -> bf16 padded to 256" if cfg4 else
                         "config 2: FixedWidth f32[256] -> bf16"),
            "h2d": h2d, "decode": decode, "verify": args.verify,
            "model": f"MLP 256-{args.hidden}-{args.hidden}-{args.hidden}-16 bf16, AdamW, batch {B}",
            "model_tflops_per_step": round(flops / 1e12, 4),
            "prestaged_ms_per_step": [round(a1, 4), round(a2, 4)],
            "loader_ms_per_step": [round(b1, 4), round(b2, 4)],
            "overhead_pct": round(sum(ovh) / 2, 2),
            "overhead_pct_pairs": [round(v, 2) for v in ovh],
            "model_tflops_prestaged": round(flops / (min(a1, a2) * 1e-3) / 1e12, 1),
            "commits": st1["commits"] + st2["commits"],
            "loader_records_per_s_in_loop": round(B / (min(b1, b2) * 1e-3), 1),
            "verify_wait_us_per_batch": round((st1.get("verify_wait_us_per_batch", 0.0)
                                               + st2.get("verify_wait_us_per_batch", 0.0)) / 2, 3),
        }
    finally:
        b.destroy()


def main():
    print(json.dumps(run(parse())))


if __name__ == "__main__":
    main()
