#!/usr/bin/env python3
"""bf16 GEMM throughput on a CU-masked HIP stream (hipExtStreamCreateWithCUMask).

Question for the loader/training split: if the training job runs on a stream that leaves k CUs
to the data path, what does its GEMM lose?  hipBLASLt's large-GEMM kernels launch one persistent
workgroup per CU (profiles/r05_s2_priority: 256 workgroups, 256 VGPRs, 65 KiB LDS), so a masked
stream can cost k/256 (dynamic tile fetch) or up to 2x (static tiles, a second wave).

Usage: python tools/probes/cumask_probe.py [--n 8192] [--reserve 0,8,16,32]
"""
import argparse
import ctypes
import json

import torch


def masked_stream(hip, n_cu: int, reserved: list[int]):
    words = (n_cu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for cu in range(n_cu):
        if cu not in reserved:
            mask[cu // 32] |= 1 << (cu % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return s


def time_gemm(a, b, c, stream, n_iter=30):
    with torch.cuda.stream(stream):
        for _ in range(3):
            torch.matmul(a, b, out=c)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n_iter):
            torch.matmul(a, b, out=c)
        e.record()
    e.synchronize()
    return s.elapsed_time(e) / n_iter


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--reserve", default="0,4,8,16,32")
    args = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    n = args.n
    a = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    flops = 2.0 * n ** 3
    out = {"n_cu": n_cu, "gemm": n}
    base = time_gemm(a, b, c, torch.cuda.current_stream())
    out["full_stream_ms"] = round(base, 4)
    out["full_tflops"] = round(flops / base / 1e9, 1)
    for k in [int(x) for x in args.reserve.split(",")]:
        for layout in ("spread", "low"):
            if k == 0 and layout == "low":
                continue
            res = ([i * (n_cu // k) for i in range(k)] if layout == "spread" else list(range(k))) if k else []
            st = torch.cuda.ExternalStream(masked_stream(hip, n_cu, res).value, device=dev)
            ms = time_gemm(a, b, c, st)
            out[f"reserve{k}_{layout}"] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1),
                                           "vs_full": round(base / ms, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
