"""The scenario of tests/test_gpu_teardown.py: close one loader while the user's stream holds
~400 ms of queued work and a second loader keeps delivering.  Importable (the test runs it in its
own process, deferred releases on) and runnable as a child (argv: broker url; the test starts it
with TORCHKAFKA_DEFERRED_FREE=0, the old inline releases, for comparison).  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def scenario(url: str, tag: str) -> dict:
    import torch

    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
    from torchkafka_amd.ops import hip

    class Vec(KafkaDataset):
        schema = FixedWidth(torch.float32, (256,))

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)

    def loader(group, h2d):
        return DeviceLoader(Vec.placeholder(), 256, num_workers=2, device=dev, dtype=torch.bfloat16, h2d=h2d,
                            decode="device",
                            worker_init_fn=Vec.init_worker("t", bootstrap_servers=url, group_id=f"{tag}-{group}",
                                                           auto_offset_reset="earliest", consumer_timeout_ms=2000))

    a, b = loader("a", "dma"), loader("b", "zerocopy")  # A has an HBM mirror, copy streams, pinned logs
    ia, ib = iter(auto_commit(a)), iter(auto_commit(b))
    for _ in range(20):
        next(ia)
        next(ib)
    torch.cuda.synchronize()
    # calibrate the user's kernel: torch.cuda._sleep(cycles)
    user = torch.cuda.Stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(user):
        e0.record()
        torch.cuda._sleep(10_000_000)
        e1.record()
    e1.synchronize()
    cycles_per_ms = 10_000_000 / e0.elapsed_time(e1)
    # the training job's queued work: 40 kernels of ~10 ms on its stream
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
    with torch.cuda.stream(user):
        evs[0].record()
        for k in range(40):
            torch.cuda._sleep(int(cycles_per_ms * 10))
            evs[k + 1].record()
    t0 = time.perf_counter()
    ia.close()
    a.close()
    close_ms = (time.perf_counter() - t0) * 1e3
    user_done_at_close = evs[-1].query()
    # the other loader keeps delivering while the user's work runs
    got, t1 = 0, time.perf_counter()
    while got < 50 and not evs[-1].query():
        x = next(ib)
        got += 1
    b_ms = (time.perf_counter() - t1) * 1e3
    user_done_after_b = evs[-1].query()
    evs[-1].synchronize()
    user_ms = evs[0].elapsed_time(evs[-1])
    gaps = [evs[k].elapsed_time(evs[k + 1]) for k in range(40)]
    ib.close()
    b.close()
    drained = bool(hip().reaper_drain(60000))
    return {"tag": tag, "close_ms": round(close_ms, 2), "user_ms": round(user_ms, 2),
            "user_kernel_ms_max": round(max(gaps), 2), "user_kernel_ms_min": round(min(gaps), 2),
            "user_done_at_close": bool(user_done_at_close), "b_batches_during_user_work": got,
            "b_ms": round(b_ms, 2), "user_done_after_b": bool(user_done_after_b),
            "reaper": dict(hip().reaper_stats()), "reaper_drained": drained,
            "last_b_batch": [list(x.shape), str(x.dtype)] if got else None}


if __name__ == "__main__":
    print(json.dumps(scenario(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "child")), flush=True)
