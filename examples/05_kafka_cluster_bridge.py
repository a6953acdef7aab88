#!/usr/bin/env python3
"""A Kafka cluster on the device path, written exactly as for the reference.

The workers are pointed at a Kafka cluster (``bootstrap_servers="host:port"``).  The DeviceLoader
mirrors this rank's partitions through a native KafkaBridge (Kafka wire protocol, C++ fetch
threads receiving each Fetch response straight into a local replica log) and decodes them on the
GPU; every batch's commit reaches the cluster's group coordinator.

No cluster is reachable here, so this example starts one: a `KafkaWireServer` serving a synthetic
broker over the Kafka protocol on 127.0.0.1.  Point ``SERVERS`` at a real cluster (whose topic
holds float32[256] records, uncompressed or gzip/snappy/lz4) to use it instead.

    python examples/05_kafka_cluster_bridge.py            # cuda:0 when available, else CPU
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torchkafka import DeviceLoader, FixedWidth, KafkaDataset, auto_commit  # noqa: E402
from torchkafka_amd.broker import KafkaWireServer, SyntheticBroker  # noqa: E402


class Features(KafkaDataset):
    schema = FixedWidth(torch.float32, (256,))


def main() -> None:
    # --- a stand-in cluster: 4 partitions x 5000 records behind the Kafka protocol
    cluster = SyntheticBroker.create(f"shm://example5-{os.getpid()}")
    cluster.create_topic("features", 4)
    cluster.fill("features", 5000, "fixed_f32", size=256)
    server = KafkaWireServer(cluster).start()
    servers = os.environ.get("SERVERS", server.address)
    try:
        device = "cuda:0" if torch.cuda.is_available() else "cpu"
        loader = DeviceLoader(Features.placeholder(), 256, num_workers=2, device=device,
                              dtype=torch.bfloat16 if device != "cpu" else torch.float32,
                              worker_init_fn=Features.init_worker("features", bootstrap_servers=servers,
                                                                  group_id="example5",
                                                                  auto_offset_reset="earliest",
                                                                  consumer_timeout_ms=1000))
        print(f"mirroring {servers} into {loader._servers} ({len(loader._bridges)} bridge)")
        n = 0
        for x in auto_commit(loader):
            n += x.shape[0]  # ... a training step on x ...
        loader.close()  # forwards the final commit to the cluster
        print(f"{n} records on {device}; the cluster's committed offsets:",
              cluster.committed_offsets("example5", "features"))
    finally:
        server.close()
        cluster.destroy()


if __name__ == "__main__":
    main()
