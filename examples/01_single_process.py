#!/usr/bin/env python3
"""Reference usage, single process (reference README.md:84-101): per-record `_process`, torch's
DataLoader, `auto_commit` commits each batch once the next one is requested.

Runs against the built-in synthetic broker (no Kafka cluster needed):
    python examples/01_single_process.py
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
        x = torch.frombuffer(bytearray(record.value), dtype=torch.float32)
        return None if x[0] % 10 == 0 else x  # None skips the record (it is still committed)


def main():
    url = f"shm://example1-{os.getpid()}"
    broker = SyntheticBroker.create(url)
    try:
        broker.create_topic("vectors", 1)
        broker.fill("vectors", 100, "fixed_f32", size=8)
        ds = Vectors("vectors", bootstrap_servers=url, group_id="example", auto_offset_reset="earliest",
                     consumer_timeout_ms=200)
        n = 0
        for batch in auto_commit(DataLoader(ds, batch_size=4)):
            n += batch.shape[0]
        print(f"consumed {n} records; committed offsets: {broker.committed_offsets('example', 'vectors')}")
    finally:
        broker.destroy()


if __name__ == "__main__":
    main()
