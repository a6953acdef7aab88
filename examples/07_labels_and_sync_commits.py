#!/usr/bin/env python3
"""(features, label) batches with coordinator-durable commits, over the Kafka protocol.

Two things the reference does with plain kafka-python and a DataLoader, on the device path:

* the label comes from the record itself -- here its key -- and rides with the values:
  ``FixedWidth(...) + Key()`` makes every batch a ``(values, labels)`` pair, the int64 key column
  decoded next to the values (on a GPU by the same kernel that checks the CRC and casts the values);
* ``commit="sync"``: batch k's OffsetCommit is answered by the group coordinator before batch
  k+1 is handed out, as the reference's ``consumer.commit()`` after every batch
  (/root/reference/src/auto_commit.py:55-58).  The default, ``"async"``, forwards the offsets
  within 5 ms instead.

No cluster is reachable here, so the example serves a synthetic broker over the Kafka protocol
(the C++ ``NativeWireServer``, Kafka 4.x version profile: the client negotiates its versions).

    python examples/07_labels_and_sync_commits.py        # cuda:0 when available, else CPU
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torchkafka import DeviceLoader, FixedWidth, KafkaDataset, Key, auto_commit  # noqa: E402
from torchkafka_amd.broker import NativeWireServer, SyntheticBroker  # noqa: E402


class Labelled(KafkaDataset):
    # 64 float32 values per record; its 8-byte big-endian key is the label
    schema = FixedWidth(torch.float32, (64,)) + Key()


def main() -> None:
    cluster = SyntheticBroker.create(f"shm://example7-{os.getpid()}")
    cluster.create_topic("events", 2)
    cluster.fill("events", 2000, "fixed_f32", size=64, keyed=True)  # key = offset % 1000
    server = NativeWireServer(cluster, profile="kafka4").start()
    try:
        device = "cuda:0" if torch.cuda.is_available() else "cpu"
        loader = DeviceLoader(Labelled.placeholder(), 128, num_workers=2, device=device, commit="sync",
                              worker_init_fn=Labelled.init_worker("events", bootstrap_servers=server.address,
                                                                  group_id="example7",
                                                                  auto_offset_reset="earliest",
                                                                  consumer_timeout_ms=1000))
        n, bad = 0, 0
        for values, labels in auto_commit(loader):
            # column 0 of each record holds its offset: the key the broker wrote is offset % 1000
            bad += int((labels != values[:, 0].long() % 1000).sum())
            n += values.shape[0]
        st = loader.stats_summary()
        loader.close()
        print(f"{n} labelled records on {device}, {bad} label mismatches; "
              f"{st['sync_commits']} synchronous commits (p99 {st['sync_commit_p99_us']:.0f} us)")
        print("the coordinator's committed offsets:", cluster.committed_offsets("example7", "events"))
    finally:
        server.close()
        cluster.destroy()


if __name__ == "__main__":
    main()
