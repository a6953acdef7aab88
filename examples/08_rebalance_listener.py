#!/usr/bin/env python3
"""A ConsumerRebalanceListener on the reference's multi-worker API.

The reference lets a subclass override ``new_consumer`` (/root/reference/README.md:46-57); with
kafka-python that is where a ``ConsumerRebalanceListener`` is attached.  Here two DataLoader
workers of one process are members of one consumer group; each worker's listener prints what it
gives up and receives.  The group forms, then a second process-like member (a plain consumer in
this process's main thread) joins and later leaves: the workers hear ``on_partitions_revoked``
(after the batches the user finished were committed) and ``on_partitions_assigned`` each time.

    python examples/08_rebalance_listener.py
"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.utils.data import DataLoader, get_worker_info  # noqa: E402

from torchkafka import ConsumerRebalanceListener, FixedWidth, KafkaConsumer, KafkaDataset, auto_commit  # noqa: E402
from torchkafka_amd.broker import SyntheticBroker  # noqa: E402


class Announce(ConsumerRebalanceListener):
    def __init__(self):
        info = get_worker_info()
        self.who = f"worker {info.id}" if info is not None else "main"

    def on_partitions_revoked(self, revoked):
        print(f"{self.who}: revoked {sorted(tp.partition for tp in revoked)}", flush=True)

    def on_partitions_assigned(self, assigned):
        print(f"{self.who}: assigned {sorted(tp.partition for tp in assigned)}", flush=True)


class Vectors(KafkaDataset):
    schema = FixedWidth(torch.float32, (8,))

    @classmethod
    def new_consumer(cls, *args, **kwargs):
        consumer = super(cls, cls).new_consumer(*args, **kwargs)
        consumer.subscribe(list(args), listener=Announce())  # re-subscribe with the listener
        return consumer


def main() -> None:
    url = f"shm://example8-{os.getpid()}"
    broker = SyntheticBroker.create(url, group_initial_rebalance_delay_ms=500)
    broker.create_topic("events", 4)
    broker.fill("events", 3000, "fixed_f32", size=8, records_per_batch=50)
    try:
        kw = dict(bootstrap_servers=url, group_id="trainer", auto_offset_reset="earliest", consumer_timeout_ms=2500)
        dl = DataLoader(Vectors.placeholder(), batch_size=64, num_workers=2, worker_init_fn=Vectors.init_worker(
            "events", **kw))

        def visitor():  # another member joins for a moment, then leaves
            time.sleep(0.8)
            c = KafkaConsumer(**{**kw, "enable_auto_commit": False})
            c.subscribe(["events"], listener=Announce())
            t0 = time.monotonic()
            while time.monotonic() - t0 < 1.0:
                c.poll(timeout_ms=20)
            c.close()

        th = threading.Thread(target=visitor)
        th.start()
        n = 0
        for batch in auto_commit(dl):
            n += batch.shape[0]
            time.sleep(0.01)  # the user's step
        th.join()
        print(f"{n} records delivered; committed {broker.committed_offsets('trainer', 'events')}")
    finally:
        broker.destroy()


if __name__ == "__main__":
    main()
