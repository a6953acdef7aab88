"""One process of tests/test_rebalance_listener.py: the reference's multi-worker API (placeholder +
init_worker + DataLoader + auto_commit) with a ConsumerRebalanceListener attached in an overridden
new_consumer (reference README.md:46-57).  The worker's listener writes every callback -- with the
group's committed offsets at that moment and the offsets of the batches the user had finished --
to a JSON file.  argv: broker url, output path."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from torchkafka_amd import ConsumerRebalanceListener, FixedWidth, KafkaDataset, auto_commit  # noqa: E402
from torchkafka_amd.broker.synthetic import open_broker  # noqa: E402

URL, OUT = sys.argv[1], sys.argv[2]
FINISHED = OUT + ".finished"  # the main process's view: offsets of the batches the user finished


class Listener(ConsumerRebalanceListener):
    def __init__(self):
        self.events = []

    def _log(self, kind, tps):
        b = open_broker(URL)
        committed = {str(p): o for p, o in b.committed_offsets("gl", "t").items() if o is not None}
        try:
            finished = json.load(open(FINISHED))
        except (OSError, ValueError):
            finished = {}
        self.events.append({"kind": kind, "tps": sorted(tp.partition for tp in tps), "committed": committed,
                            "finished": finished})
        with open(OUT, "w") as f:
            json.dump({"events": self.events}, f)

    def on_partitions_revoked(self, revoked):
        self._log("revoked", revoked)

    def on_partitions_assigned(self, assigned):
        self._log("assigned", assigned)


class Vec(KafkaDataset):
    schema = FixedWidth(torch.float32, (4,))

    @classmethod
    def new_consumer(cls, *args, **kwargs):
        c = super(cls, cls).new_consumer(*args, **kwargs)
        c.subscribe(list(args), listener=Listener())
        return c


def main():
    dl = DataLoader(Vec.placeholder(), batch_size=10, num_workers=1,
                    worker_init_fn=Vec.init_worker("t", bootstrap_servers=URL, group_id="gl",
                                                   auto_offset_reset="earliest", consumer_timeout_ms=3000))
    finished = {}
    n = 0
    for x in auto_commit(dl):
        # the previous batches are finished once this one is handed out; record this one's ends
        # for the next step (what the worker must have committed by a revocation after it)
        with open(FINISHED + ".tmp", "w") as f:
            json.dump(finished, f)
        os.replace(FINISHED + ".tmp", FINISHED)
        for o, p in x[:, :2].tolist():
            finished[str(int(p))] = max(finished.get(str(int(p)), 0), int(o) + 1)
        n += 1
        if n == 3:
            open(OUT + ".ready", "w").close()
        time.sleep(0.02)


if __name__ == "__main__":
    main()
