#!/usr/bin/env python3
"""The ``_process``-override path (VERDICT r4 "do this" 7): the reference README's own dataset.

The reference's documented usage subclasses KafkaDataset with a ``_process`` of its own that
parses each record's JSON (/root/reference/README.md:72-79, ``json.loads(record.value)``).  Such a
dataset cannot use the native header walk or the device decoders: every record goes through the
user's Python.  This block measures that path on config 4's records (JSON arrays of 16..256
numbers, ~1 KiB of text), ``_process = torch.tensor(json.loads(record.value))``, 4 workers, batch
256, per-batch commit, two ways over the same topic (a consumer group each):

* ``device_loader``: ``DeviceLoader`` -- the workers run ``_process`` per record (the reference's
  per-record loop, loader/worker.py ``_generic_loop``), pack the variable-length rows into a ring
  slot, and the device pads + stacks them (a 1-D var-len batch -> ``(B, max_len)`` f32 on the GPU);
* ``torch_dataloader``: ``torch.utils.data.DataLoader(dataset, batch_size=256, num_workers=4,
  pin_memory=True, collate_fn=pad_sequence)`` + ``.cuda(non_blocking=True)`` -- what a user of
  the reference writes (variable-length lists fail ``default_collate``, SURVEY B25, so a padding
  collate is required), committed by the same ``auto_commit``.

Both deliver the same padded f32 batches on the GPU.

Usage: python benchmarks/process_override.py [--steps K] [--device cuda:0]
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
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--min-len", type=int, default=16)
    ap.add_argument("--max-len", type=int, default=256)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--modes", default="device_loader,torch_dataloader")
    return ap.parse_args(argv)


def _readme_dataset():
    import torch

    from torchkafka_amd import KafkaDataset

    class ReadmeJson(KafkaDataset):
        """The reference README's dataset: one tensor of the record's JSON array."""

        def _process(self, record):
            return torch.tensor(json.loads(record.value))

    return ReadmeJson


# at module level so DataLoader workers can pickle it
def pad_collate(batch):
    from torch.nn.utils.rnn import pad_sequence

    return pad_sequence(batch, batch_first=True)


def _time(it, steps, warmup, to_device, sync):
    import torch

    x = None
    for _ in range(warmup):
        x = to_device(next(it))
    if x is not None and x.is_cuda:
        torch.cuda.synchronize()
    if sync is not None:
        sync()
    t0 = time.perf_counter()
    rows = 0
    for _ in range(steps):
        x = to_device(next(it))
        rows += x.shape[0]
    if x.is_cuda:
        torch.cuda.synchronize()
    if sync is not None:
        sync()
    return rows, time.perf_counter() - t0, x


def run(args, sync=None) -> dict:
    import torch
    from torch.utils.data import DataLoader

    from torchkafka_amd import DeviceLoader, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    ReadmeJson = _readme_dataset()
    url = f"shm://tkproc-{os.getpid()}"
    b = SyntheticBroker.create(url, log_capacity=1 << 32)
    modes = [m for m in args.modes.split(",") if m]
    out = {"metric": "records/s to GPU through a user _process (json.loads), per-batch commit",
           "dataset": "README MyDataset: _process = torch.tensor(json.loads(record.value))",
           "records": f"JSON arrays of {args.min_len}..{args.max_len} numbers (config 4)",
           "batch_size": args.batch_size, "workers": args.workers, "partitions": args.partitions,
           "steps": args.steps}
    try:
        b.create_topic("json", args.partitions)
        B = args.batch_size
        per_part = int(math.ceil((args.steps + args.warmup + 16 * args.workers) * B * 1.2 / args.partitions))
        b.fill("json", per_part, "json_f32", size=args.min_len, max_size=args.max_len, threads=args.partitions)
        dev = torch.device(args.device)
        kw = dict(bootstrap_servers=url, auto_offset_reset="earliest", consumer_timeout_ms=2000)
        for mode in modes:
            if mode == "device_loader":
                dl = DeviceLoader(ReadmeJson.placeholder(), B, num_workers=args.workers, device=dev,
                                  dtype=torch.float32,
                                  worker_init_fn=ReadmeJson.init_worker("json", group_id="proc-dl", **kw))
                it = iter(auto_commit(dl))
                rows, el, x = _time(it, args.steps, args.warmup, lambda v: v[0] if isinstance(v, tuple) else v, sync)
                path = dl.plan.describe() if hasattr(dl.plan, "describe") else None
                it.close()
                dl.close()
            elif mode == "torch_dataloader":
                dl = DataLoader(ReadmeJson.placeholder(), batch_size=B, num_workers=args.workers,
                                pin_memory=dev.type == "cuda", collate_fn=pad_collate, prefetch_factor=4,
                                worker_init_fn=ReadmeJson.init_worker("json", group_id="proc-torch", **kw))
                it = iter(auto_commit(dl))
                rows, el, x = _time(it, args.steps, args.warmup, lambda v: v.to(dev, non_blocking=True), sync)
                path = ("torch DataLoader(num_workers, pin_memory=True, collate_fn=pad_sequence) + "
                        ".cuda(non_blocking=True)")
                it.close()
                del dl
            else:
                raise ValueError(f"unknown mode {mode}")
            out[mode] = {"records_per_s": round(rows / el, 1), "ms_per_step": round(el / args.steps * 1e3, 4),
                         "timed_s": round(el, 4), "last_batch": [list(x.shape), str(x.dtype), str(x.device)],
                         **({"path": path} if path else {})}
        if "device_loader" in out and "torch_dataloader" in out:
            out["device_loader_vs_torch"] = round(out["device_loader"]["records_per_s"]
                                                  / out["torch_dataloader"]["records_per_s"], 3)
        return out
    finally:
        b.destroy()


def main():
    print(json.dumps(run(parse())))


if __name__ == "__main__":
    main()
