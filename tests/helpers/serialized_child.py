"""One process of tests/test_gpu_serialized.py: the fixed-width, var-len, JSON and HBM-mirror
loaders over one broker, each into a consumer group of its own (named by `tag`), every delivered
tensor digested in order.  Run with or without AMD_SERIALIZE_KERNEL / AMD_SERIALIZE_COPY /
HIP_LAUNCH_BLOCKING (read at HIP start-up, hence a process of its own) and TORCHKAFKA_HIP_QUEUE.

argv: broker url, tag.  Prints one JSON line: {loader: {"digest", "rows", "committed"}}.
"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from torchkafka_amd import DeviceLoader, FixedWidth, JsonArray, KafkaDataset, VarLen, auto_commit  # noqa: E402
from torchkafka_amd.broker.synthetic import open_broker  # noqa: E402


def main() -> None:
    url, tag = sys.argv[1], sys.argv[2]
    dev = sys.argv[3] if len(sys.argv) > 3 else "cuda:0"  # "cpu": a host rehearsal of the helper
    b = open_broker(url)
    cases = {
        "fixed": ("fixed", FixedWidth(torch.float32, (64,)), dict(dtype=torch.bfloat16)),
        "varlen": ("tokens", VarLen(torch.int32, max_len=48), dict(dtype=torch.int64, pad_value=-1)),
        "json": ("json", JsonArray(max_len=40), dict(dtype=torch.bfloat16)),
        "mirror": ("fixed", FixedWidth(torch.float32, (64,)), dict(dtype=torch.bfloat16, h2d="dma")),
    }
    out = {}
    for name, (topic, schema, kw) in cases.items():
        if dev == "cpu":
            kw = {k: v for k, v in kw.items() if k != "h2d"}
        else:
            kw = {**kw, "decode": "device"}
        ds_cls = type(f"DS_{name}", (KafkaDataset,), {"schema": schema})
        group = f"{tag}-{name}"
        dl = DeviceLoader(ds_cls.placeholder(), 48, num_workers=2, device=dev, in_order=True,
                          worker_init_fn=ds_cls.init_worker(topic, bootstrap_servers=url, group_id=group,
                                                            auto_offset_reset="earliest", consumer_timeout_ms=500),
                          **kw)
        h, rows = hashlib.sha256(), 0
        for x in auto_commit(dl):
            for t in (x if isinstance(x, (tuple, list)) else (x,)):
                if isinstance(t, torch.Tensor):
                    h.update(t.detach().cpu().contiguous().view(torch.uint8).numpy().tobytes())
            rows += (x[0] if isinstance(x, (tuple, list)) else x).shape[0]
        dl.close()
        out[name] = {"digest": h.hexdigest(), "rows": rows,
                     "committed": {str(k): v for k, v in sorted(b.committed_offsets(group, topic).items())}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
