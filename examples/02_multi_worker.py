#!/usr/bin/env python3
"""Reference usage with DataLoader workers (reference README.md:103-132): a placeholder dataset,
one consumer per worker built by `init_worker`, and exact per-worker commits (this framework's
fix of the reference's prefetch overshoot).

    python examples/02_multi_worker.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from torchkafka import KafkaDataset, auto_commit  # noqa: E402
from torchkafka_amd.broker import SyntheticBroker  # noqa: E402


class Vectors(KafkaDataset):
    def _process(self, record):
        return torch.frombuffer(bytearray(record.value), dtype=torch.float32)


def main():
    url = f"shm://example2-{os.getpid()}"
    broker = SyntheticBroker.create(url)
    try:
        broker.create_topic("vectors", 4)
        broker.fill("vectors", 200, "fixed_f32", size=8)
        dl = DataLoader(Vectors.placeholder(), batch_size=16, num_workers=2,
                        worker_init_fn=Vectors.init_worker("vectors", bootstrap_servers=url, group_id="example",
                                                           auto_offset_reset="earliest", consumer_timeout_ms=300))
        n = sum(batch.shape[0] for batch in auto_commit(dl))
        print(f"consumed {n} records; committed offsets: {broker.committed_offsets('example', 'vectors')}")
    finally:
        broker.destroy()


if __name__ == "__main__":
    main()
