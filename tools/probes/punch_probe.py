"""Probe: which host-memory operations stall the GPU of the calling process?

A replica log that is pinned (hipHostRegister) in chunks and then released (unpin, then
fallocate(PUNCH_HOLE)) showed ~170 ms GPU stalls.  This probe keeps a stream of small kernels
running, performs one operation at a time on a shm file mapped in this process, and reports the
largest gap between consecutive kernel completions around it.
"""
import ctypes
import mmap
import os
import threading
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
libc = ctypes.CDLL("libc.so.6", use_errno=True)
MB = 1 << 20
path = f"/dev/shm/punch_probe_{os.getpid()}"
fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o666)
N = 1024 * MB
os.ftruncate(fd, N)
m = mmap.mmap(fd, N)
buf = (ctypes.c_char * N).from_buffer(m)
base = ctypes.addressof(buf)
for i in range(0, N, MB):
    m[i:i + 8] = b"xxxxxxxx"  # touch one byte per 4K? fill whole pages below
m.seek(0)
chunk = b"y" * MB
for i in range(0, N, MB):
    m[i:i + MB] = chunk


def reg(off, n):
    assert hip.hipHostRegister(ctypes.c_void_p(base + off), ctypes.c_size_t(n), ctypes.c_uint(2)) == 0


def unreg(off):
    assert hip.hipHostUnregister(ctypes.c_void_p(base + off)) == 0


def punch(off, n):
    assert libc.fallocate(fd, 3, ctypes.c_long(off), ctypes.c_long(n)) == 0


def dontneed(off, n):
    assert libc.madvise(ctypes.c_void_p(base + off), ctypes.c_size_t(n), 4) == 0  # MADV_DONTNEED


torch.cuda.init()
x = torch.ones(1 << 20, device="cuda")
gaps = []
stop = threading.Event()


def spin():
    ev = [torch.cuda.Event() for _ in range(2)]
    last = time.perf_counter()
    while not stop.is_set():
        x.mul_(1.0000001)
        torch.cuda.synchronize()
        now = time.perf_counter()
        gaps.append((now, now - last))
        last = now


def measure(label, fn):
    gaps.clear()
    t0 = time.perf_counter()
    time.sleep(0.05)
    fn()
    time.sleep(0.3)
    worst = max(g for t, g in gaps if t > t0)
    print(f"{label:60s} max kernel gap {worst * 1e3:8.2f} ms")


th = threading.Thread(target=spin, daemon=True)
th.start()
time.sleep(0.2)
measure("baseline (nothing)", lambda: None)
reg(0, 64 * MB)
reg(64 * MB, 64 * MB)
measure("register 64 MiB", lambda: reg(128 * MB, 64 * MB))
measure("unregister 64 MiB", lambda: unreg(128 * MB))
measure("punch 64 MiB never registered, mapped here", lambda: punch(512 * MB, 64 * MB))
measure("punch 64 MiB previously registered (unregistered)", lambda: punch(128 * MB, 64 * MB))
measure("punch 2 MiB inside a REGISTERED chunk", lambda: punch(2 * MB, 2 * MB))
measure("madvise(DONTNEED) 64 MiB never registered", lambda: dontneed(600 * MB, 64 * MB))
unreg(64 * MB)
measure("dontneed+punch 64 MiB after unregister", lambda: (dontneed(64 * MB, 64 * MB), punch(64 * MB, 64 * MB)))
stop.set()
th.join()
unreg(0)
os.close(fd)
os.unlink(path)
