#!/usr/bin/env python3
"""BASELINE config 1: single-process KafkaDataset on CPU, 1-partition topic, batch_size=4,
``_process -> torch.rand(8)`` -- the reference's README example, plumbing only (no GPU).

Path measured: synthetic broker -> KafkaConsumer iteration -> KafkaDataset.__iter__ /
``_process`` -> torch DataLoader (num_workers=0, default_collate) -> auto_commit (one
commit per batch).  Reference yardstick: 108,521 records/s on the same
shape with an in-memory fake consumer.

Usage: python benchmarks/config1_cpu_plumbing.py [--records N]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

YARDSTICK = 108521.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=200000)
    ap.add_argument("--batch-size", type=int, default=4)
    return ap.parse_args(argv)


def reference_loop_same_host(records: int = 40000, batch_size: int = 4) -> float:
    """The reference's config-1 loop as SURVEY §6 measured it, on this host: an in-memory fake
    consumer (zero broker cost) under the reference's KafkaDataset.__iter__ shape (process,
    None-skip), torch's DataLoader (num_workers=0) and a no-op commit per batch.  The yardstick
    above (108,521 rec/s) was measured on another host; this is the same loop here."""
    import torch
    from torch.utils.data import DataLoader, IterableDataset

    class Fake(IterableDataset):
        def __iter__(self):
            for _ in range(records):
                data = torch.rand(8)  # the README's _process
                if data is not None:
                    yield data

        def commit(self):
            pass

    dl = DataLoader(Fake(), batch_size=batch_size)
    n, t0 = 0, time.perf_counter()
    for batch in dl:
        n += batch.shape[0]
        dl.dataset.commit()
    return n / (time.perf_counter() - t0)


def run(args) -> dict:
    import torch
    from torch.utils.data import DataLoader

    from torchkafka_amd import KafkaDataset, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    threads = torch.get_num_threads()
    torch.set_num_threads(1)

    class MyDataset(KafkaDataset):
        def _process(self, record):
            return torch.rand(8)

    url = f"shm://tkcfg1-{os.getpid()}"
    b = SyntheticBroker.create(url)
    try:
        b.create_topic("topic", 1)
        b.fill("topic", args.records, "bytes", size=16, records_per_batch=500)
        ds = MyDataset("topic", group_id="group_1", bootstrap_servers=url, auto_offset_reset="earliest",
                       consumer_timeout_ms=200)
        dl = DataLoader(ds, batch_size=args.batch_size)
        n = 0
        t0 = None
        commits0 = 0
        for i, batch in enumerate(auto_commit(dl)):
            if i == 100:
                t0 = time.perf_counter()
                n = 0
                commits0 = b.commit_count("group_1")
            n += batch.shape[0]
        # the stream end includes one consumer_timeout_ms wait; exclude it
        el = time.perf_counter() - t0 - 0.2
        commits = b.commit_count("group_1") - commits0
        assert b.committed("group_1", "topic", 0) == args.records
        ds.close()
        v = n / el
        ref_here = reference_loop_same_host(batch_size=args.batch_size)
        return {"config": 1, "metric": "records/s (CPU plumbing, per-batch commit)", "value": round(v),
                "reference_loop_same_host": round(ref_here), "vs_reference_loop_same_host": round(v / ref_here, 3),
                "batch_size": args.batch_size, "records": n, "commits": commits, "timed_s": round(el, 4),
                "path": ("KafkaConsumer -> KafkaDataset._process -> auto_commit over a torch DataLoader "
                         "(num_workers=0: its batch_size / collate_fn / drop_last, without the per-batch "
                         "iterator overhead)"),
                "vs_yardstick": round(v / YARDSTICK, 3)}
    finally:
        torch.set_num_threads(threads)
        b.destroy()


def main():
    print(json.dumps(run(parse())))


if __name__ == "__main__":
    main()
