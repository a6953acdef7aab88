"""Worker fill cost per batch on the host, by pack kind (no GPU): RecordBatch walk + CRC32C +
pack of one ring slot, as a DeviceLoader worker does it.  Usage: python tools/fill_bench.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(kind_name, gen, size, max_size, bs=256, batches=300, check_crcs=True):
    from torchkafka_amd.broker import SyntheticBroker
    from torchkafka_amd.ops.native import core

    c = core()
    url = f"shm://tkfill-{os.getpid()}-{kind_name}"
    b = SyntheticBroker.create(url, log_capacity=1 << 31)
    try:
        b.create_topic("t", 1)
        b.fill("t", bs * (batches + 4), gen, size=size, max_size=max_size)
        ring = c.Ring.create(f"/tkfillring-{os.getpid()}", 1, 2, 16 << 20)
        try:
            f = c.Fetcher(b.native, check_crcs)
            f.assign([b.topic("t")[0]], [0])
            kind = getattr(c, kind_name)
            elem, row = (4, size) if kind == c.PACK_FIXED else (4, 0)
            ts = []
            for i in range(batches):
                g = i % 2
                ring.worker_acquire(0, g, 1000)
                t0 = time.perf_counter_ns()
                f.fill_slot(ring, g, kind, elem, row, 0, -1, True, False, bs, 100, False)
                ts.append(time.perf_counter_ns() - t0)
                ring.worker_publish(g)
                assert ring.main_acquire(100) == g
                ring.main_release(g)
            ts.sort()
            return {"kind": kind_name, "us_per_batch_p50": round(ts[len(ts) // 2] / 1e3, 1),
                    "us_per_batch_min": round(ts[0] / 1e3, 1)}
        finally:
            ring.shutdown()
            ring.unlink()
    finally:
        b.destroy()


def main():
    out = [bench("PACK_FIXED", "fixed_f32", 256, 0), bench("PACK_JSON_F32", "json_f32", 16, 256),
           bench("PACK_JSON_TEXT", "json_f32", 16, 256)]
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
