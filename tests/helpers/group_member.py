"""One consumer process of tests/test_group_rebalance.py: the reference's API (KafkaDataset +
DataLoader + auto_commit) against a Kafka-protocol test cluster, as a member of group "g".

argv: bootstrap address, num_workers, seconds to sleep per batch, idle timeout (ms)[, "device"].
"device": a DeviceLoader (device="cpu", bridge=False) whose workers are the group members and read
the replica with the native fetch loop.
Prints one JSON line: every (partition, offset) the loop received, in order.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from torchkafka_amd import FixedWidth, KafkaDataset, auto_commit  # noqa: E402


class Vec(KafkaDataset):
    schema = FixedWidth(torch.float32, (8,))


def main() -> None:
    addr, nw, slow, idle = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
    kw = dict(bootstrap_servers=addr, group_id="g", auto_offset_reset="earliest", consumer_timeout_ms=idle,
              heartbeat_interval_ms=100, session_timeout_ms=6000)
    if len(sys.argv) > 5 and sys.argv[5] == "device":
        from torchkafka_amd import DeviceLoader

        dl = DeviceLoader(Vec.placeholder(), 8, device="cpu", num_workers=nw, bridge=False,
                          worker_init_fn=Vec.init_worker("t", **kw))
    elif nw == 0:
        dl = DataLoader(Vec("t", **kw), batch_size=8)
    else:
        dl = DataLoader(Vec.placeholder(), batch_size=8, num_workers=nw, worker_init_fn=Vec.init_worker("t", **kw))
    seen = []
    for x in auto_commit(dl):
        seen += [(int(p), int(o)) for o, p in x[:, :2].tolist()]
        if slow:
            time.sleep(slow)
    print(json.dumps({"seen": seen}), flush=True)


if __name__ == "__main__":
    main()
