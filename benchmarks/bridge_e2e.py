#!/usr/bin/env python3
"""A Kafka cluster over TCP -> KafkaBridge replica -> DeviceLoader (device decode) -> commits back.

Not a BASELINE config: it measures the production route of `KafkaBridge` on the config-2 record
shape (f32[256], 1 KiB records, batch 256, commit after every batch).  The cluster is
`NativeWireServer` (C++, record sets sent from the mapped logs; `--python-server`: the Python
`KafkaWireServer`) over a synthetic broker, one server process per node (partition p led by node
p % nodes) on the loopback interface, so the numbers include the Kafka protocol, TCP, the
replicator's fetch threads (one per leader) and its commit forwarding; they do not include a real
broker's disk or a NIC.

Phases: (1) replication alone: a backlog mirrored from the cluster into the replica (GB/s);
(2) end to end: a fresh group replicates and consumes concurrently, every batch's offsets
committed locally and forwarded to the cluster (records/s), and the cluster's committed offsets are
checked at the end.

Usage: python benchmarks/bridge_e2e.py [--nodes 4 --partitions 8 --records 200000]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _SkipCluster(Exception):
    pass


def _free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def _serve(url, node_id, cluster, ready, python_server):
    from torchkafka_amd.broker import KafkaWireServer, NativeWireServer, open_broker

    cls = KafkaWireServer if python_server else NativeWireServer
    srv = cls(open_broker(url), port=cluster[node_id][2], node_id=node_id, cluster=cluster).start()
    ready.set()
    while True:
        time.sleep(3600)
    srv.close()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--records", type=int, default=500_000, help="records per partition")
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--partition-fetch-mib", type=int, default=8)
    ap.add_argument("--max-lag-mib", type=int, default=512)
    ap.add_argument("--release-mib", type=int, default=256, help="consumed bytes kept resident per partition")
    ap.add_argument("--ring-mib", type=int, default=512, help="replica ring per partition (0: linear + release)")
    ap.add_argument("--release-step-mib", type=int, default=1024, help="release burst threshold per partition")
    ap.add_argument("--no-release", action="store_true", help="keep committed replica bytes (no unpin/punch)")
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--unpin-only", action="store_true",
                    help="experiment: the device driver unpins consumed ranges, the replicator frees nothing")
    ap.add_argument("--numa", action="store_true", help="bind to the GPU's NUMA node before filling/replicating")
    ap.add_argument("--h2d", default="auto", choices=["auto", "dma", "zerocopy"])
    ap.add_argument("--direct", action="store_true",
                    help="control run: phase 2 consumes the cluster's own broker directly (no wire, no replica)")
    ap.add_argument("--python-server", action="store_true",
                    help="serve the cluster with the Python KafkaWireServer instead of the native one")
    ap.add_argument("--no-cluster", action="store_true", help="control: no servers, no bridge (implies --direct)")
    ap.add_argument("--backlog", action="store_true",
                    help="phase 2 waits until the replica holds the whole backlog before consuming it (the "
                         "consumer side alone)")
    args = ap.parse_args()
    if args.no_cluster:
        args.direct, args.nodes = True, 0

    from torchkafka_amd.broker import KafkaBridge, SyntheticBroker

    if args.numa and args.device.startswith("cuda"):
        from torchkafka_amd.utils.topology import bind_to_gpu_numa

        bind_to_gpu_numa(int(args.device.split(":")[1]) if ":" in args.device else 0)
    url = f"shm://tkbe2e-{os.getpid()}"
    src = SyntheticBroker.create(url, log_capacity=1 << 34, index_capacity=1 << 22)
    src.create_topic("t", args.partitions)
    t0 = time.perf_counter()
    src.fill("t", args.records, "fixed_f32", size=args.dim, records_per_batch=64, threads=min(16, args.partitions))
    fill_s = time.perf_counter() - t0
    total_bytes = sum(src.native.log_bytes(src.pidx("t", p)) for p in range(args.partitions))
    ports = _free_ports(args.nodes)
    cluster = [(i, "127.0.0.1", ports[i]) for i in range(args.nodes)]
    ctx = mp.get_context("fork")  # before any HIP call in this process
    procs = []
    for i in range(args.nodes):
        ev = ctx.Event()
        pr = ctx.Process(target=_serve, args=(url, i, cluster, ev, args.python_server), daemon=True)
        pr.start()
        ev.wait(30)
        procs.append(pr)
    boot = f"127.0.0.1:{ports[0]}" if ports else None
    out = {"server": "python" if args.python_server else "native", "nodes": args.nodes,
           "partitions": args.partitions, "records_per_partition": args.records,
           "cluster_gb": round(total_bytes / 1e9, 3), "fill_s": round(fill_s, 2)}
    try:
        # (1) replication alone
        if args.no_cluster:
            raise _SkipCluster
        t0 = time.perf_counter()
        br = KafkaBridge(boot, "t", url=f"shm://tkbe2e-r-{os.getpid()}", log_capacity=1 << 34,
                         index_capacity=1 << 22, max_partition_fetch_bytes=args.partition_fetch_mib << 20,
                         max_lag_bytes=1 << 40)
        ok = br.wait_caught_up(300)
        rep_s = time.perf_counter() - t0
        out["replication"] = {"caught_up": ok, "s": round(rep_s, 3), "gb_per_s": round(total_bytes / rep_s / 1e9, 2),
                              "fetch_threads": br._r.fetch_threads,
                              "errors": br.errors}
        br.close()
    except _SkipCluster:
        pass
    try:
        # (2) end to end: replicate + decode + commit concurrently
        import torch

        from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit

        class Rows(KafkaDataset):
            schema = FixedWidth(torch.float32, (args.dim,))

        dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
        br = None if args.no_cluster else KafkaBridge(
                         boot, "t", group_id="trainer", url=f"shm://tkbe2e-e-{os.getpid()}", log_capacity=1 << 34,
                         index_capacity=1 << 22, max_partition_fetch_bytes=args.partition_fetch_mib << 20,
                         max_lag_bytes=args.max_lag_mib << 20,
                         release_consumed=not (args.no_release or args.unpin_only),
                         release_bytes=args.release_mib << 20, release_step=args.release_step_mib << 20,
                         ring_bytes=args.ring_mib << 20)
        if br is not None and args.unpin_only:
            br.local.native.flags = 1  # kReleaseConsumed: the driver unpins, nobody punches
        dl = DeviceLoader(Rows.placeholder(), args.batch_size, num_workers=args.workers, device=args.device,
                          dtype=dtype, h2d=args.h2d,
                          worker_init_fn=Rows.init_worker("t", bootstrap_servers=url if args.direct else br.url,
                                                                       group_id="trainer",
                                                                       auto_offset_reset="earliest",
                                                                       consumer_timeout_ms=2000))
        import threading

        caught = {}

        def _watch():
            caught["ok"] = br.wait_caught_up(300)
            caught["t"] = time.perf_counter()

        if br is None:
            pass
        elif args.backlog:
            _watch()
        else:
            threading.Thread(target=_watch, daemon=True).start()
        n = n_first = 0
        t0 = time.perf_counter()
        t_first = t_last = None
        marks = []
        for x in auto_commit(dl):
            n += x.shape[0]
            t_last = time.perf_counter()
            marks.append((t_last, n))
            if t_first is None:  # worker fork + HIP init + first fetches are startup, not throughput
                t_first, n_first = t_last, n
        if args.device.startswith("cuda"):
            torch.cuda.synchronize()
        # A worker's last, partial batch is only handed over after its consumer timeout (the end
        # of a stream is a timeout): the timed region ends at the last batch before that stall.
        for (ta, na), (tb, _nb) in zip(marks, marks[1:]):
            if tb - ta > 0.5:
                t_last, n = ta, na
                break
        el = t_last - t_first
        out["startup_to_first_batch_s"] = round(t_first - t0, 3)
        if "t" in caught and not args.backlog:
            out["replica_caught_up_after_first_batch_s"] = round(caught["t"] - t_first, 3)
        if args.stats:
            print(json.dumps({"loader": dl.stats_summary(), "bridge": br.stats() if br else None}), file=sys.stderr)
        n_timed = n - n_first
        if br is not None:
            br.close()
        committed = src.committed_offsets("trainer", "t")
        if args.direct:
            committed = {p: args.records for p in committed}  # committed straight into the source
        out["end_to_end"] = {"records": n, "records_total": marks[-1][1], "s": round(el, 3),
                             "records_per_s": round(n_timed / el, 1),
                             "gb_per_s": round(n_timed * args.dim * 4 / el / 1e9, 2),
                             "decode": "device" if dl.plan.span else "host",
                             "cluster_committed_ok": all(v == args.records for v in committed.values()),
                             "loader": {k: v for k, v in dl.stats_summary().items()
                                        if k in ("worker_fill_us_per_batch", "commit_latency_p99_us",
                                                 "log_mib_unpinned")}}
    finally:
        for pr in procs:
            pr.terminate()
        src.destroy()
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
