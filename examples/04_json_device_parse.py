#!/usr/bin/env python3
"""JSON records decoded on the GPU: the reference README's `json.loads(record.value)` dataset,
as a `JsonArray` schema.

The workers only frame each record (element count + a streaming copy of the text into the
pinned ring); the gfx950 `json_rows_kernel` parses the numbers, pads the batch to its longest
row and casts to bf16, bit-exact with `json.loads` + `torch.tensor(..., float32).to(bf16)`.
Rows shorter than `min_len` are skipped like the reference's `_process -> None` and are still
committed. A malformed row stops the loop with `CorruptRecordException` before its batch is
committed, so a restart re-reads it.

    python examples/04_json_device_parse.py            # cuda:0 if present, else the CPU path
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torchkafka import DeviceLoader, JsonArray, KafkaDataset, auto_commit  # noqa: E402
from torchkafka_amd.broker import SyntheticBroker  # noqa: E402
from torchkafka_amd.client.producer import KafkaProducer  # noqa: E402


class Sequences(KafkaDataset):
    schema = JsonArray(min_len=2)  # `[..]` of numbers -> float32 row; shorter rows are skipped


def main():
    url = f"shm://example4-{os.getpid()}"
    broker = SyntheticBroker.create(url)
    try:
        broker.create_topic("seq", 4)
        producer = KafkaProducer(bootstrap_servers=url, value_serializer=lambda v: json.dumps(v).encode())
        for i in range(2000):
            producer.send("seq", value=[round(0.25 * (i % 97) - j, 2) for j in range(i % 40)], partition=i % 4)
        producer.flush()
        device = "cuda:0" if torch.cuda.is_available() else "cpu"
        loader = DeviceLoader(Sequences.placeholder(), 128, num_workers=2, device=device, dtype=torch.bfloat16,
                              return_mask=True,
                              worker_init_fn=Sequences.init_worker("seq", bootstrap_servers=url, group_id="ex4",
                                                                   auto_offset_reset="earliest",
                                                                   consumer_timeout_ms=500))
        rows = 0
        for x, lengths, mask in auto_commit(loader):  # x: [128, L] bf16, L = the batch's longest row
            rows += x.shape[0]
            assert bool((mask.sum(1) == lengths).all())
        print(f"{rows} rows on {device} (device parse: {loader.plan.json_device}); "
              f"committed {broker.committed_offsets('ex4', 'seq')}")
    finally:
        broker.destroy()


if __name__ == "__main__":
    main()
