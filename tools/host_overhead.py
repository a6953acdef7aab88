"""Host-side cost of each call on the DeviceLoader per-batch path (run on the GPU box)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=20000):
    fn()
    t0 = time.perf_counter_ns()
    for _ in range(n):
        fn()
    return (time.perf_counter_ns() - t0) / n


def main():
    import torch

    from torchkafka_amd.ops import hip

    res = {k: round(v, 1) for k, v in hip().api_bench(0, 20000)}
    dev = torch.device("cuda", 0)
    res["torch.empty((256,256),bf16,cuda)"] = round(
        timeit(lambda: torch.empty((256, 256), dtype=torch.bfloat16, device=dev)), 1)
    res["torch._C._cuda_getCurrentRawStream"] = round(timeit(lambda: torch._C._cuda_getCurrentRawStream(0)), 1)
    res["torch.cuda.current_stream().cuda_stream"] = round(
        timeit(lambda: torch.cuda.current_stream(dev).cuda_stream), 1)
    x = torch.empty(1, device=dev)
    res["Tensor.data_ptr()"] = round(timeit(lambda: x.data_ptr()), 1)
    print(json.dumps({"host_ns_per_call": res}, indent=1))


if __name__ == "__main__":
    main()
