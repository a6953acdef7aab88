#!/usr/bin/env python3
"""Which HIP teardown calls wait for an unrelated stream's work?  

A loader's close() must not stall the user's training stream.  This probe queues a ~200 ms spin
kernel on a torch stream, then times each teardown call the loader's native code makes (on
memory of its own, through libamdhip64 via ctypes).  A call that takes ~200 ms waited for the
unrelated kernel (a device-wide synchronisation).

Usage: python tools/probes/sync_probe.py   (on a GPU box)
"""
import ctypes
import json
import time

import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    torch.zeros(1, device=dev)
    st = torch.cuda.Stream(dev)
    own = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(own), 1) == 0
    cycles = int(2.1e9 * 0.2)  # ~200 ms of spinning

    def timed(name, fn):
        with torch.cuda.stream(st):
            torch.cuda._sleep(cycles)
        time.sleep(0.005)  # the spin kernel is running
        t = time.perf_counter()
        rc = fn()
        ms = (time.perf_counter() - t) * 1e3
        torch.cuda.synchronize()
        return name, {"rc": rc, "ms": round(ms, 2)}

    out = {}
    for name, make, free in [
        ("hipFree", lambda p: hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)), lambda p: hip.hipFree(p)),
        ("hipFreeAsync(own stream)", lambda p: hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)),
         lambda p: hip.hipFreeAsync(p, own)),
        ("hipHostFree", lambda p: hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20), 0),
         lambda p: hip.hipHostFree(p)),
    ]:
        p = ctypes.c_void_p()
        assert make(p) == 0
        k, v = timed(name, lambda: free(p))
        out[k] = v
    buf = ctypes.create_string_buffer(1 << 22)
    assert hip.hipHostRegister(ctypes.cast(buf, ctypes.c_void_p), ctypes.c_size_t(1 << 22), 0) == 0
    k, v = timed("hipHostUnregister", lambda: hip.hipHostUnregister(ctypes.cast(buf, ctypes.c_void_p)))
    out[k] = v
    k, v = timed("hipStreamSynchronize(own)", lambda: hip.hipStreamSynchronize(own))
    out[k] = v
    ev = ctypes.c_void_p()
    hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)
    k, v = timed("hipEventDestroy", lambda: hip.hipEventDestroy(ev))
    out[k] = v
    s2 = ctypes.c_void_p()
    hip.hipStreamCreateWithFlags(ctypes.byref(s2), 1)
    k, v = timed("hipStreamDestroy(idle own)", lambda: hip.hipStreamDestroy(s2))
    out[k] = v
    k, v = timed("hipDeviceSynchronize", lambda: hip.hipDeviceSynchronize())
    out[k] = v
    print(json.dumps({"sync_probe_ms_with_200ms_kernel_on_another_stream": out}))


if __name__ == "__main__":
    main()
