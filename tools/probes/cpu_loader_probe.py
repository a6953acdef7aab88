"""DeviceLoader(device='cpu') throughput on the config-2 record shape (the CPU fallback path)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit  # noqa: E402
from torchkafka_amd.broker import SyntheticBroker  # noqa: E402


class Rows(KafkaDataset):
    schema = FixedWidth(torch.float32, (256,))


url = f"shm://tkcdl-{os.getpid()}"
src = SyntheticBroker.create(url, log_capacity=1 << 30)
src.create_topic("t", 8)
src.fill("t", 40000, "fixed_f32", size=256, threads=8)
for workers in (2, 4):
    dl = DeviceLoader(Rows.placeholder(), 256, num_workers=workers, device="cpu",
                      worker_init_fn=Rows.init_worker("t", bootstrap_servers=url, group_id=f"g{workers}",
                                                      auto_offset_reset="earliest", consumer_timeout_ms=1000))
    n, t_first, marks = 0, None, []
    for x in auto_commit(dl):
        n += x.shape[0]
        marks.append((time.perf_counter(), n))
    end = len(marks) - 1
    for i in range(1, len(marks)):
        if marks[i][0] - marks[i - 1][0] > 0.5:
            end = i - 1
            break
    el = marks[end][0] - marks[0][0]
    st = dl.stats_summary()
    print(f"workers {workers}: {(marks[end][1] - marks[0][1]) / el / 1e6:.2f} M rec/s "
          f"(host wait {st['host_wait_us_per_batch']:.0f} us, issue {st['host_issue_us_per_batch']:.0f} us per batch)")
    dl.close()
src.destroy()
