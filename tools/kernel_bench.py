#!/usr/bin/env python3
"""Device-resident throughput of the gfx950 collate kernels vs PyTorch's own kernels.

Inputs already live in HBM, so this measures the kernels alone (the loader's H2D is
measured by bench.py).  For each case it prints the device time per call (``gpu_us``:
calls captured in a HIP graph and replayed, so host launch cost is excluded) and the
effective HBM bandwidth (bytes read + bytes written) / time, next to the equivalent
PyTorch op (``Tensor.to`` for the cast, an index_put-based pad for var-len); ``eager_us``
is the wall time per eager call including the Python wrapper and launch.

Usage: python tools/kernel_bench.py [--quick] [--iters N]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    import torch

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters  # µs


def timeit_graph(fn, iters, per_graph=20):
    """Device time per call: `per_graph` calls captured in one HIP graph, replayed, so the host's
    per-launch cost (Python wrapper + hipLaunchKernel) is out of the measurement."""
    import torch

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn()
    g.replay()
    torch.cuda.synchronize()
    reps = max(1, iters // per_graph)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1000.0 / (reps * per_graph)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="fewer iterations (for counter collection)")
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    iters = 20 if args.quick else args.iters

    import torch

    from torchkafka_amd.ops.collate import collate_fixed, collate_varlen
    from torchkafka_amd.ops.native import hip

    hip()
    dev = torch.device("cuda", 0)
    out = []

    fixed_cases = [("config2 batch 256x256 f32->bf16", 256, 256, torch.bfloat16),
                   ("256x256 f32->fp8e4m3", 256, 256, torch.float8_e4m3fn),
                   ("bs1024 1024x256 f32->bf16", 1024, 256, torch.bfloat16),
                   ("config5 8x262144 f32->bf16 (8 MiB)", 8, 262144, torch.bfloat16),
                   ("64x262144 f32->bf16 (64 MiB)", 64, 262144, torch.bfloat16),
                   ("256x262144 f32->bf16 (256 MiB)", 256, 262144, torch.bfloat16)]
    for name, rows, row, dt in fixed_cases:
        src = torch.randn(rows, row, device=dev)
        t_ours = timeit(lambda: collate_fixed(src, dt), iters)
        t_torch = timeit(lambda: src.to(dt), iters)
        g_ours = timeit_graph(lambda: collate_fixed(src, dt), iters)
        g_torch = timeit_graph(lambda: src.to(dt), iters)
        nbytes = src.numel() * 4 + src.numel() * torch.empty((), dtype=dt).element_size()
        out.append({"kernel": "fixed", "case": name, "gpu_us": round(g_ours, 2),
                    "GBps": round(nbytes / g_ours / 1e3, 1),
                    "torch_gpu_us": round(g_torch, 2), "torch_GBps": round(nbytes / g_torch / 1e3, 1),
                    "eager_us": round(t_ours, 2), "torch_eager_us": round(t_torch, 2)})

    g = torch.Generator().manual_seed(0)
    var_cases = [("config4 256 rows, L~U(0,512) f32->bf16", 256, 512, torch.float32),
                 ("256 rows, L~U(0,8192) f32->bf16", 256, 8192, torch.float32),
                 ("4096 rows, L~U(0,4096) f32->bf16", 4096, 4096, torch.float32),
                 ("LDS-staged: 4096 rows, L~U(0,4096) bf16->bf16", 4096, 4096, torch.bfloat16)]
    src_code = {torch.float32: 0, torch.bfloat16: 2}
    for name, rows, lmax, sdt in var_cases:
        lens = torch.randint(0, lmax + 1, (rows,), generator=g)
        offs = torch.zeros(rows + 1, dtype=torch.int32)
        offs[1:] = lens.cumsum(0).to(torch.int32)
        vals = torch.randn(int(offs[-1]), device=dev).to(sdt)
        offs_d = offs.to(dev)
        L = int(lens.max())
        esz = vals.element_size()
        nbytes = vals.numel() * esz + rows * L * 2

        buf = torch.zeros(vals.numel() * esz + 64, dtype=torch.uint8, device=dev)
        buf[: vals.numel() * esz].copy_(vals.view(torch.uint8))
        o = torch.empty((rows, L), dtype=torch.bfloat16, device=dev)
        ln = torch.empty(rows, dtype=torch.int64, device=dev)
        mod = hip()
        stream = torch.cuda.current_stream(dev).cuda_stream

        def ours():
            mod.collate_varlen(offs_d.data_ptr(), buf.data_ptr(), src_code[sdt], o.data_ptr(), 2, rows, L, 0.0,
                               ln.data_ptr(), 0, stream)

        row_idx = torch.repeat_interleave(torch.arange(rows, device=dev), lens.to(dev))
        col_idx = torch.arange(vals.numel(), device=dev) - offs_d[:-1].long().repeat_interleave(lens.to(dev))

        def torch_pad():
            t = torch.zeros((rows, L), dtype=torch.bfloat16, device=dev)
            t[row_idx, col_idx] = vals.to(torch.bfloat16)
            return t

        # numerics check once
        ours()
        assert torch.equal(o.view(torch.int16), torch_pad().view(torch.int16))
        _ = collate_varlen(offs_d, vals, torch.bfloat16, L=L)
        t_ours = timeit(ours, iters)
        t_torch = timeit(torch_pad, iters)
        g_ours = timeit_graph(lambda: mod.collate_varlen(offs_d.data_ptr(), buf.data_ptr(), src_code[sdt], o.data_ptr(),
                                                          2, rows, L, 0.0, ln.data_ptr(), 0,
                                                          torch.cuda.current_stream(dev).cuda_stream), iters)
        g_torch = timeit_graph(torch_pad, iters)
        out.append({"kernel": "varlen", "case": name, "gpu_us": round(g_ours, 2),
                    "GBps": round(nbytes / g_ours / 1e3, 1),
                    "torch_gpu_us": round(g_torch, 2), "torch_GBps": round(nbytes / g_torch / 1e3, 1),
                    "eager_us": round(t_ours, 2), "torch_eager_us": round(t_torch, 2)})

    # device JSON parse (json_parse.hip) from HBM: text bytes parsed per second, against the
    # workers' native host parser on the same rows (no PyTorch GPU equivalent exists)
    import random
    import time

    import numpy as np

    from torchkafka_amd.ops.native import core

    rnd = random.Random(0)
    for name, rows in (("config4 256 rows JSON -> bf16", 256), ("4096 rows JSON -> bf16", 4096)):
        texts = []
        for _ in range(rows):
            n = rnd.randint(16, 256)
            texts.append(("[" + ", ".join("%.2f" % rnd.uniform(-50, 51) for _ in range(n)) + "]").encode())
        desc = np.zeros((rows, 4), dtype=np.int32)
        blob = bytearray()
        for i, t in enumerate(texts):
            at = (len(blob) + 31) // 32 * 32
            blob.extend(b"\0" * (at - len(blob)))
            cnt = core().json_scan_simple(t)
            desc[i] = (at, len(t), cnt, cnt)
            blob.extend(t)
        blob.extend(b"\0" * 64)
        L = int(desc[:, 3].max())
        d_desc = torch.from_numpy(desc).to(dev)
        d_vals = torch.frombuffer(blob, dtype=torch.uint8).to(dev)
        o = torch.empty((rows, L), dtype=torch.bfloat16, device=dev)
        ln = torch.empty(rows, dtype=torch.int64, device=dev)
        mod = hip()

        def jparse():
            mod.launch_json_rows(d_desc.data_ptr(), d_vals.data_ptr(), o.data_ptr(), 2, rows, L, 0.0, ln.data_ptr(), 0,
                                 0, torch.cuda.current_stream(dev).cuda_stream)

        jparse()
        ref = torch.zeros((rows, L), dtype=torch.float32)
        for i, t in enumerate(texts):
            v = json.loads(t)
            ref[i, : len(v)] = torch.tensor(v, dtype=torch.float64).float()
        assert torch.equal(o.cpu().view(torch.int16), ref.to(torch.bfloat16).view(torch.int16))
        g_ours = timeit_graph(jparse, iters)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            for t in texts:
                core().parse_json_f32(t)
        host_us = (time.perf_counter() - t0) / reps * 1e6
        text_bytes = sum(len(t) for t in texts)
        out.append({"kernel": "json_parse", "case": name, "gpu_us": round(g_ours, 2),
                    "text_GBps": round(text_bytes / g_ours / 1e3, 1), "numbers": int(desc[:, 2].sum()),
                    "host_parser_us_one_core": round(host_us, 1)})

    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
