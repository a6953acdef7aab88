"""Host time of each step in 20-step windows after a synchronize, and the final drain (fixed-width, 1 GPU)."""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
from torchkafka_amd.broker import SyntheticBroker
class R(KafkaDataset):
    schema = FixedWidth(torch.float32, (256,))
url = f"shm://probe-{os.getpid()}"
b = SyntheticBroker.create(url, log_capacity=1 << 32)
b.create_topic("t", 8); b.fill("t", 40000, "fixed_f32", size=256, threads=8)
dl = DeviceLoader(R.placeholder(), 256, num_workers=4, device="cuda:0", dtype=torch.bfloat16,
                  worker_init_fn=R.init_worker("t", bootstrap_servers=url, group_id="g", auto_offset_reset="earliest"))
it = iter(auto_commit(dl))
for _ in range(5): next(it)
for rep in range(5):
    torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for _ in range(20):
        s = time.perf_counter(); next(it); ts.append((time.perf_counter() - s) * 1e6)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"steps_us": [round(x, 1) for x in ts], "loop_us": round((t1 - t0) * 1e6, 1),
                      "sync_us": round((t2 - t1) * 1e6, 1)}), flush=True)
it.close(); dl.close(); b.destroy()
