#!/usr/bin/env python3
"""The Kafka-protocol bridge alone, without a loader: how fast a KafkaBridge ring replica mirrors a
topic served by the C++ wire server, uncompressed and compressed, when the consumer side is free
(a thread commits the replica's end as fast as it grows).  Isolates fetch + inflate + ingest from
the device decode (bench.py's bridge_<codec> blocks measure them together).

    python tools/probes/bridge_probe.py [--records 100000] [--partitions 8] [--codecs none,lz4,zstd]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=100000, help="records per partition")
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--codecs", default="none,lz4,zstd")
    ap.add_argument("--max-partition-fetch-mib", type=int, default=8)
    ap.add_argument("--fetchers", type=int, default=0)
    a = ap.parse_args()
    from torchkafka_amd.broker import KafkaBridge, NativeWireServer, SyntheticBroker
    from torchkafka_amd.client.records import TopicPartition

    b = SyntheticBroker.create(f"shm://tkbprobe-{os.getpid()}", log_capacity=1 << 32, index_capacity=1 << 22)
    srv = None
    out = {}
    try:
        b.create_topic("src", a.partitions)
        b.fill("src", a.records, "fixed_f32", size=a.dim, records_per_batch=64, threads=a.partitions)
        srv = NativeWireServer(b, profile="kafka4").start()
        for codec in a.codecs.split(","):
            topic = f"t_{codec}"
            b.create_topic(topic, a.partitions)
            info = b.copy_compressed("src", topic, None if codec == "none" else codec)
            br = KafkaBridge(srv.address, topic, group_id=f"g_{codec}",
                             max_partition_fetch_bytes=a.max_partition_fetch_mib << 20, fetchers=a.fetchers,
                             start=False)
            done = threading.Event()

            def consume():  # the replica's consumer: commits its end as soon as it grows
                parts = [TopicPartition(topic, p) for p in range(a.partitions)]
                while not done.is_set():
                    ends = {tp: br.local.end_offset(topic, tp.partition) for tp in parts}
                    br.local.commit(f"g_{codec}", {tp: e for tp, e in ends.items() if e > 0})
                    time.sleep(0.0002)

            th = threading.Thread(target=consume, daemon=True)
            t0 = time.perf_counter()
            br.start()
            th.start()
            while any(br.local.end_offset(topic, p) < a.records for p in range(a.partitions)):
                time.sleep(0.001)
            el = time.perf_counter() - t0
            done.set()
            th.join()
            st = br.stats()
            tot = {k: sum(int(s[k]) for s in st) for k in ("wire_bytes", "recv_ns", "ingest_ns", "inflate_ns",
                                                             "inflated_bytes", "fetches", "throttled")}
            thr = int(br._r.fetch_threads)
            inf = max(1, int(br._r.inflate_threads) or thr)
            out[codec] = {"records_per_s": round(a.records * a.partitions / el, 1), "s": round(el, 3),
                          "raw_gb_per_s": round(info["raw_bytes"] / el / 1e9, 2),
                          "wire_gb_per_s": round(tot["wire_bytes"] / el / 1e9, 2),
                          "ratio": round(info["raw_bytes"] / max(1, info["compressed_bytes"]), 2),
                          "fetch_threads": thr, "inflate_threads": int(br._r.inflate_threads),
                          "fetches": tot["fetches"], "throttled": tot["throttled"],
                          "share": {"fetch_wait": round(int(br._r.fetch_wait_ns) / 1e9 / (thr * el), 3),
                                    "recv": round(tot["recv_ns"] / 1e9 / (thr * el), 3),
                                    "inflate": round(tot["inflate_ns"] / 1e9 / (inf * el), 3),
                                    "ingest": round(tot["ingest_ns"] / 1e9 / (inf * el), 3)},
                          "errors": br.errors}
            print(codec, json.dumps(out[codec]), flush=True)
            br.close()
    finally:
        if srv is not None:
            srv.close()
        b.destroy()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
