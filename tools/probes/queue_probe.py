#!/usr/bin/env python3
"""Which HIP streams share a hardware queue?  (the lockstep stream's queue.)

A process gets GPU_MAX_HW_QUEUES (4) hardware queues per priority; HIP binds streams to them as
they are created.  Two streams on one queue serialise: a kernel on one waits behind the other's.
This probe makes `--normal` normal-priority streams and one stream at the device's greatest
priority, parks a ~60 ms spin kernel on every normal stream (and the default stream), then times
a tiny kernel on each stream: ~60 ms means it waited behind a spin kernel on a shared queue.

Usage: python tools/probes/queue_probe.py [--normal 5]
"""
import argparse
import ctypes
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--normal", type=int, default=5)
    ap.add_argument("--high-pool", type=int, default=4,
                    help="then: spin on this many high-priority streams, probe one more")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    torch.zeros(1, device=dev)
    lo, hi = torch.cuda.Stream.priority_range()  # (least, greatest)
    normal = [torch.cuda.Stream(dev) for _ in range(args.normal)]
    high = torch.cuda.Stream(dev, priority=hi)
    hip = ctypes.CDLL("libamdhip64.so")
    raw = ctypes.c_void_p()
    hip.hipStreamCreateWithFlags(ctypes.byref(raw), 1)  # a raw non-blocking stream, as the loader makes them
    raw_s = torch.cuda.ExternalStream(raw.value, device=dev)
    # touch every stream once (HIP binds a stream to a queue at first use)
    for s in [*normal, high, raw_s]:
        with torch.cuda.stream(s):
            torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    cycles = int(2.1e9 * 0.06)
    spin_on = [torch.cuda.default_stream(dev), *normal]
    for s in spin_on:
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
    time.sleep(0.002)
    out = {"priority_range": [lo, hi], "normal_streams": args.normal}

    def probe(name, s):
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            ev = torch.cuda.Event()
            torch.cuda._sleep(100)
            ev.record()
        ev.synchronize()
        out[name] = round((time.perf_counter() - t0) * 1e3, 2)

    probe("high_priority_stream_ms", high)
    probe("raw_nonblocking_stream_ms", raw_s)
    torch.cuda.synchronize()
    # the high-priority pool's size: busy high-priority streams, then one more
    highs = [torch.cuda.Stream(dev, priority=hi) for _ in range(args.high_pool + 1)]
    for s in highs:
        with torch.cuda.stream(s):
            torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    for s in highs[:-1]:
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
    time.sleep(0.002)
    probe(f"high_priority_stream_after_{args.high_pool}_busy_high_ms", highs[-1])
    probe("normal_stream_while_high_busy_ms", normal[0])
    torch.cuda.synchronize()
    print(json.dumps({"queue_probe": out}))


if __name__ == "__main__":
    main()
