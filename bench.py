#!/usr/bin/env python3
"""Headline benchmark: Kafka records/sec delivered to the GPU with a commit after every batch.

BASELINE.json metric "Kafka records/sec to GPU with per-batch commit, at
1/2/4/8 MI355X".  Configurations (BASELINE.json ``configs``):

  * N = 1 : config 2 -- 1x MI355X, num_workers=4, 8-partition topic,
            fixed-width float32 records (256 x f32 = 1 KiB), pinned ring +
            hipMemcpyAsync on a side stream, gfx950 collate kernel -> bf16;
  * N > 1 : config 3 -- one process per GPU, 8 partitions per rank
            (64 at N = 8), static rank sharding, auto_commit lock-stepped by an
            RCCL all-reduce over xGMI every step.

A step = one batch of ``--batch-size`` records per rank consumed from the
synthetic broker, decoded on the GPU (CRC32C + values cast to bf16 by the
gfx950 kernels), handed to the user, and its offsets committed (the commit of
batch k happens when batch k+1 is requested, as in the reference's
auto_commit, /root/reference/src/auto_commit.py:55-58).  Records are synthetic
Kafka RecordBatch v2 records (an 8-byte key, the offset % 1000, and 1 KiB of
float32 values each) produced into the shared-memory broker before timing (a
retained backlog).  Weak scaling: per-rank work is fixed as N grows.

Launch: ``python bench.py --gpus N --steps K --warmup W``.  Under torchrun
(``WORLD_SIZE`` set) this process is one rank.  Without it and N > 1, this
process starts N rank processes itself -- before any GPU call, as fresh
children with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 set --
relays rank 0's single JSON line and exits with the first failing rank's code.
It refuses to run (exit 2) when fewer than N GPUs are visible.

Blocks in the one JSON line (all timed between a barrier + synchronize on both
sides, max over ranks, whole-job records):
  * ``value``: the driver's K steps (after W warm-up steps);
  * ``steady_state``: ``--steady-steps`` more steps of the same loader (default
    50 000: >= 0.25 s at the measured rate; the workers' prefilled slots are a
    fraction of a percent of it), with per-rank rates and the lockstep's cost;
  * ``steady_dma``: a second loader (own consumer group, same topic from the
    earliest offset) with ``h2d="dma"``: the partition logs are copied into HBM
    by hipMemcpyAsync on a side stream (SDMA) and decoded there -- the config-2
    mechanism;
  * ``steady_f32``: a third loader delivering float32 (the reference's dtype);
  * ``steady_label``: values plus the record key as an int64 label column per batch
    (``FixedWidth(...) + Key()``: the worker reads each key while it walks the headers, the decode
    kernel copies the labels beside the values) -- ``(features, label)`` batches;
  * ``bridge``: the same records served over the Kafka protocol (a native C++ wire server on the
    loopback interface, Kafka 4.x version profile) to a DeviceLoader whose KafkaBridge mirrors this
    rank's partitions into a local ring replica and forwards every commit to the group
    coordinator -- ``async`` (the default commit mode; coordinator round trips reported) and
    ``sync`` (``commit="sync"``: batch k's OffsetCommit answered before batch k+1 is handed out).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import threading
import time

BASELINE_METRIC = "Kafka records/sec to GPU with per-batch commit, at 1/2/4/8 MI355X"
# reference measured on config 2's shape without a GPU (bs=256, 1 KiB f32[256], nw=4)
BASELINE_VALUE = 337237.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--dim", type=int, default=256, help="float32 elements per record")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--partitions-per-gpu", type=int, default=8)
    ap.add_argument("--slots-per-worker", type=int, default=None, help="ring depth (default: loader's auto)")
    ap.add_argument("--prefetch", type=int, default=2)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "f16", "f32"])
    ap.add_argument("--records-per-batch", type=int, default=64, help="Kafka RecordBatch size in the log")
    ap.add_argument("--no-crc", action="store_true", help="skip CRC32C verification (kafka-python check_crcs)")
    ap.add_argument("--device", default=None, help="override device (e.g. cpu for a dry run)")
    ap.add_argument("--stats", action="store_true", help="print loader stats to stderr")
    ap.add_argument("--window-trace", type=int, default=0,
                    help="diagnostic: after the headline, time this many more headline-sized windows step by "
                         "step and print where their time goes to stderr")
    ap.add_argument("--in-order", action="store_true", help="strict worker round-robin delivery")
    ap.add_argument("--event-every", type=int, default=None)
    ap.add_argument("--h2d", default="auto", choices=["auto", "dma", "zerocopy", "direct"])
    ap.add_argument("--copy-streams", type=int, default=4)
    ap.add_argument("--mirror-chunk-mib", type=int, default=8,
                    help="--h2d dma with device decode: MiB per hipMemcpyAsync into the HBM log mirror")
    ap.add_argument("--mirror-chunks", type=int, default=None, help="--h2d dma: HBM mirror buffers per partition")
    ap.add_argument("--lockstep-depth", type=int, default=None, help="default: the loader's auto depth")
    ap.add_argument("--lockstep-commit-every", type=int, default=None,
                    help="async lockstep: an agreement every n steps (default: the loader's, per transport)")
    ap.add_argument("--verify", default="deliver", choices=["deliver", "commit"],
                    help="deliver: a batch is handed out after its device CRC verdict landed (default); commit: "
                         "the verdict gates only its commit")
    ap.add_argument("--coalesce", type=int, default=None,
                    help="staged batches collated per kernel launch (default: the loader's, 6 for fixed width)")
    ap.add_argument("--coalesce-wait-us", type=int, default=50, help="adaptive coalescing wait while the GPU is busy")
    ap.add_argument("--decode-streams", type=int, default=None,
                    help="HIP streams for the device decode (default: the loader's, fitted to the hardware queues)")
    ap.add_argument("--no-numa", action="store_true", help="do not bind ranks to their GPU's NUMA node")
    ap.add_argument("--decode", default="auto", choices=["auto", "device", "host"],
                    help="device: gfx950 RecordBatch decode + CRC from the pinned logs; host: workers CRC-check + pack")
    ap.add_argument("--lockstep", default="auto", choices=["auto", "off", "rccl", "host", "shm"],
                    help="cross-rank step/commit agreement: auto = the loader's choice at N > 1 (the node-local "
                         "shared-memory transport on one host), none at N = 1; shm/rccl/host force it (also at "
                         "N = 1) over shared memory / the native RCCL communicator / the process group's all-reduce")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 with a gloo group (rehearse N > 1 ranks on a one-GPU box)")
    ap.add_argument("--steady-steps", type=int, default=None,
                    help="steps of the steady-state block timed after the headline (default: max(50 x ring "
                         "slots, 50000) on a GPU, 2000 on the CPU; 0 skips it)")
    ap.add_argument("--extra-blocks", default="dma,f32,label,shm,shm_sync,rccl,rccl_sync,verify",
                    help="comma list of secondary steady blocks, each a fresh loader over the same topic: dma "
                         "(h2d='dma', HBM mirror filled by SDMA), f32 (float32 output), label (the record key as "
                         "an int64 label beside the values: FixedWidth + Key()), shm (the node-local shared-memory "
                         "lockstep, forced also at N = 1), shm_sync (the same with commit='sync': one agreement per "
                         "step after every commit -- the cross-rank barrier), rccl / rccl_sync (the same over the "
                         "native RCCL communicator), "
                         "verify (the other --verify mode: steady_unverified or steady_verified); '' for none")
    ap.add_argument("--extra-steps", type=int, default=None,
                    help="timed steps of each secondary block (default: the steady-state steps)")
    ap.add_argument("--self-launch", action="store_true",
                    help="start the rank processes from this process even at --gpus 1 / --same-device (the "
                         "launcher path the N > 1 runs take without torchrun)")
    ap.add_argument("--config-blocks", default="train,compute,config4,config5,config1,process",
                    help="comma list of blocks run at N = 1, each on a broker of its own: train (a bf16 MLP "
                         "training step fed by auto_commit(loader) against the same step over pre-staged device "
                         "batches: the loader's cost inside a real step), compute (a bf16 GEMM "
                         "stream beside the config-2 and config-4 loaders: what the loader costs a training job), "
                         "config4 (JSON -> bf16), config5 (1 MiB records, 128 partitions), config1 (CPU plumbing), "
                         "process (the README's json.loads _process: DeviceLoader vs torch DataLoader + "
                         "pin_memory); '' for none")
    ap.add_argument("--compute-steps", type=int, default=20000)
    ap.add_argument("--train-steps", type=int, default=1500, help="timed steps per loop of the train block")
    ap.add_argument("--config4-steps", type=int, default=20000)
    ap.add_argument("--config5-steps", type=int, default=1000)
    ap.add_argument("--config1-records", type=int, default=100000)
    ap.add_argument("--process-steps", type=int, default=1500)
    ap.add_argument("--bridge-steps", type=int, default=None,
                    help="timed steps of the Kafka-protocol bridge blocks (async; sync runs a quarter): "
                         "default 8000 on a GPU, 20 on the CPU; 0 skips them")
    ap.add_argument("--bridge-codecs", default="lz4,zstd",
                    help="comma list of compressed bridge blocks (bridge_<codec>: the wire server serves the "
                         "records as compressed RecordBatches, produced while the block runs, and the bridge's "
                         "fetch threads inflate them): lz4, zstd, gzip, and <codec>_static (the whole topic "
                         "produced before the timed steps: the bridge and the decode without the producer); "
                         "'' for none")
    return ap.parse_args()


# ---------------------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """N > 1 without torchrun: start N rank processes (this process never touches the GPU --
    ``torch.cuda.device_count()`` does not initialise HIP on this image) and relay rank 0's line."""
    n = args.gpus
    parent = {}
    if not args.device:
        # counted without any HIP call (sysfs KFD topology + amdsmi): the parent must never initialise HIP
        from torchkafka_amd.utils.topology import count_gpus_without_hip, hip_touched

        try:
            gpus = count_gpus_without_hip()
        except RuntimeError as e:
            print(f"[bench] {e}: refusing to launch", file=sys.stderr)
            return 2
        parent = {"gpus_visible": gpus, **hip_touched()}
        if not args.same_device and gpus["count"] < n:
            print(f"[bench] --gpus {n} but only {gpus['count']} GPU(s) are visible ({gpus}): refusing to run "
                  "fewer ranks", file=sys.stderr)
            return 2
        if parent["torch_cuda_initialized"] or parent["kfd_fds"]:
            print(f"[bench] the launcher initialised HIP before starting its ranks ({parent}): refusing",
                  file=sys.stderr)
            return 2
    rep = os.environ.get("TK_BENCH_PARENT_REPORT")
    if rep:
        with open(rep, "w") as f:
            json.dump(parent, f)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   TK_BENCH_LAUNCHER=f"bench.py self-launch ({n} child ranks)")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    lines: list[str] = []

    def relay():
        for line in procs[0].stdout:
            lines.append(line)
            if not line.startswith('{"metric"'):
                sys.stderr.write(line)

    t = threading.Thread(target=relay, daemon=True)
    t.start()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                rc = bad[0][1]
                print(f"[bench] rank {bad[0][0]} exited with {rc}: stopping the other ranks", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    t.join(timeout=10)
    out = [x for x in lines if x.startswith('{"metric"')]
    if rc == 0:
        if len(out) != 1:
            print(f"[bench] rank 0 printed {len(out)} result lines", file=sys.stderr)
            return 1
        res = json.loads(out[0])
        if res.get("n_gpus") != n:
            print(f"[bench] rank 0 reported n_gpus={res.get('n_gpus')}, launched {n}", file=sys.stderr)
            return 1
        sys.stdout.write(out[0])
        sys.stdout.flush()
    return rc if rc >= 0 else 128 - rc


# ---------------------------------------------------------------------------------------- one rank
class Rank:
    """One rank's side of the job: process group, device, the shared broker, timing helpers."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.args = torch, dist, args
        self.rank = int(os.environ.get("RANK", 0))
        self.world = int(os.environ.get("WORLD_SIZE", 1))
        self.local_rank = int(os.environ.get("LOCAL_RANK", 0))
        if self.world != args.gpus:
            raise SystemExit(f"[bench] WORLD_SIZE={self.world} but --gpus={args.gpus}")
        dev = args.device
        if not dev:
            if not args.same_device and self.local_rank >= torch.cuda.device_count():
                raise SystemExit(f"[bench] rank {self.rank}: LOCAL_RANK {self.local_rank} but only "
                                 f"{torch.cuda.device_count()} GPU(s) visible")
            dev = f"cuda:{0 if args.same_device else self.local_rank}"
        self.device = torch.device(dev)
        self.use_gloo = self.device.type != "cuda" or args.same_device or args.lockstep == "host"

    def init_group(self) -> None:
        dist = self.dist
        if self.world > 1 or self.args.lockstep in ("rccl", "host", "shm"):
            # no GPU touched yet: the loader forks its workers before HIP is initialised
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
            dist.init_process_group("gloo" if self.use_gloo else "nccl", rank=self.rank, world_size=self.world)

    def _t(self, vals):
        torch = self.torch
        return torch.tensor(vals, dtype=torch.float64, device="cpu" if self.use_gloo else self.device)

    def barrier(self) -> None:
        if self.dist.is_initialized():
            self.dist.barrier(device_ids=[self.device.index] if not self.use_gloo else None)

    def sync(self) -> None:
        torch = self.torch
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if self.world > 1:
            self.barrier()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)

    def gather(self, vals: list[float]) -> list[list[float]]:
        """Every rank's ``vals`` (rank order)."""
        if self.world == 1:
            return [list(vals)]
        t = self._t(vals)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [[float(v) for v in x.tolist()] for x in out]

    def check_ranks(self) -> dict:
        """Start-up proof that the process group spans the job: one all-reduce of the rank ids."""
        if self.world == 1:
            return {"process_group": None, "world_size": 1}
        t = self._t([float(self.rank)])
        self.dist.all_reduce(t)
        s = int(t.item())
        want = self.world * (self.world - 1) // 2
        if s != want:
            raise RuntimeError(f"rank-id all-reduce gave {s}, expected {want} for {self.world} ranks")
        return {"process_group": self.dist.get_backend(), "world_size": self.dist.get_world_size(),
                "rank_id_sum": s}


def _thread_cpu(pids) -> dict:
    """{(pid, tid, name): cpu seconds} of every thread of ``pids`` (Linux /proc; diagnostic)."""
    out = {}
    tick = os.sysconf("SC_CLK_TCK")
    for pid in pids:
        try:
            tids = os.listdir(f"/proc/{pid}/task")
        except OSError:
            continue
        for tid in tids:
            try:
                with open(f"/proc/{pid}/task/{tid}/stat") as f:
                    s = f.read()
            except OSError:
                continue
            name = s[s.index("(") + 1:s.rindex(")")]
            f = s[s.rindex(")") + 2:].split()
            out[(pid, int(tid), name)] = (int(f[11]) + int(f[12])) / tick  # utime + stime
            out[("cpu", int(tid), name)] = int(f[36])  # the CPU it last ran on
    return out


def cpu_report(before: dict, after: dict, el: float, main_pid: int) -> dict:
    """TK_BENCH_CPU=1: the threads that used the CPU during a timed block, in cores (CPU s / wall s)."""
    last_cpu = {k[1]: v for k, v in after.items() if k[0] == "cpu"}
    after = {k: v for k, v in after.items() if k[0] != "cpu"}
    used = sorted(((after[k] - before.get(k, 0.0), k) for k in after), reverse=True)
    top = [{"who": "main" if k[0] == main_pid else "worker", "tid": k[1], "name": k[2], "cores": round(u / el, 2),
            "cpu": last_cpu.get(k[1])} for u, k in used[:12] if u > 0]
    per, by_name = {}, {}
    for u, k in used:
        w = "main" if k[0] == main_pid else "workers"
        per[w] = per.get(w, 0.0) + u
        by_name[f"{w}:{k[2]}"] = by_name.get(f"{w}:{k[2]}", 0.0) + u
    aff = {}
    for pid in sorted({k[0] for k in after}):
        try:
            aff["main" if pid == main_pid else str(pid)] = len(os.sched_getaffinity(pid))
        except OSError:
            pass
    return {"cores": {w: round(u / el, 2) for w, u in per.items()}, "threads": top,
            "by_name": {n: round(u / el, 2) for n, u in sorted(by_name.items(), key=lambda x: -x[1]) if u > 0},
            "affinity": len(os.sched_getaffinity(0)), "affinity_of": aff}


class BlockGuard:
    """Iterator wrapper for a secondary block: its first exception is kept instead of raised, and the
    loader is closed at once (a lockstep transport then leaves, so the other ranks' blocks fail
    within milliseconds instead of waiting out the lockstep timeout); next() then returns None.
    time_steps() gathers every rank's flag and raises on every rank at the same point, so the
    ranks leave a failed block with the same collectives behind them."""

    def __init__(self, it, loader):
        self.it, self.loader, self.error = it, loader, None

    def __iter__(self):
        return self

    def __next__(self):
        if self.error is not None:
            return None
        try:
            return next(self.it)
        except StopIteration:
            raise
        except Exception as e:  # noqa: BLE001 - raised by time_steps on every rank
            self.fail(e.with_traceback(None))  # (a kept traceback would keep the generator's frame alive)
            return None

    def fail(self, e: BaseException) -> None:
        self.error = e
        for close in (self.it.close, self.loader.close):  # the iteration's lockstep transport, the loader
            try:
                close()
            except Exception:  # noqa: BLE001
                pass

    def close(self) -> None:
        self.it.close()


def time_steps(R: Rank, it, steps: int, loader, trace: list | None = None) -> dict:
    """Times ``steps`` batches: barrier + synchronize on both sides, max time over ranks.
    ``trace`` (diagnostic): receives each step's end time and the closing sync's, from t0, in ns.
    TK_BENCH_CPU=1 (diagnostic): the CPU time of every thread of this process and the loader's
    workers over the block, in ``res["cpu"]``."""
    loader.reset_stats()
    R.sync()
    occ = loader.ring_occupancy()
    cpu_pids = None
    if os.environ.get("TK_BENCH_CPU") == "1":
        run = getattr(loader, "_run", None)
        cpu_pids = [os.getpid()] + [p.pid for p in getattr(run, "procs", []) if getattr(p, "pid", None)]
        cpu0 = _thread_cpu(cpu_pids)
    t0 = time.perf_counter()
    rows = 0
    x = None
    for _ in range(steps):
        x = next(it)
        if x is None:  # a BlockGuard'ed block failed on this rank
            break
        rows += (x[0] if isinstance(x, (tuple, list)) else x).shape[0]
        if trace is not None:
            trace.append(time.perf_counter() - t0)
    R.sync()
    el = time.perf_counter() - t0
    if trace is not None:
        trace.append(el)
    err = getattr(it, "error", None)
    gathered = R.gather([el, float(rows), 0.0 if err is None else 1.0])
    failed = [r for r, g in enumerate(gathered) if g[2]]
    if failed:
        raise RuntimeError(f"block failed on rank(s) {failed}"
                           + (f": {type(err).__name__}: {err}" if err is not None else ""))
    per_rank = [g[:2] for g in gathered]
    tmax = max(p[0] for p in per_rank)
    total = sum(p[1] for p in per_rank)
    st = loader.stats_summary()
    res = {"el": tmax, "rows": total, "per_rank": per_rank, "stats": st, "occ": occ, "last": x}
    if cpu_pids:
        res["cpu"] = cpu_report(cpu0, _thread_cpu(cpu_pids), el, os.getpid())
    return res


def window_trace(R: Rank, it, steps: int, n: int, loader) -> dict:
    """Diagnostic (--window-trace): ``n`` windows shaped like the headline's, each step's host time
    and the closing synchronize timed apart, and the native driver's counters over each window.
    Medians over the windows, in microseconds (counters: per window)."""
    per_step, tails, totals = [[] for _ in range(steps)], [], []
    keys = ("groups", "ahead_groups", "ahead_ns", "phase_launch_ns", "phase_next_ns", "phase_commit_ns",
            "fast_ns", "poll_ns", "blocked_ns", "verify_wait_ns", "events", "released")
    ctr = {k: [] for k in keys}
    run = getattr(loader, "_run", None)
    drv = run.driver if run is not None else None
    for _ in range(n):
        if drv is not None:
            drv.reset_stats()
        R.sync()
        t0 = t = time.perf_counter_ns()
        for k in range(steps):
            next(it)
            u = time.perf_counter_ns()
            per_step[k].append(u - t)
            t = u
        R.sync()
        u = time.perf_counter_ns()
        tails.append(u - t)
        totals.append(u - t0)
        if drv is not None:
            st = drv.stats()
            for k in keys:
                if isinstance(st.get(k, 0), (int, float)):
                    ctr[k].append(st.get(k, 0))

    def med(xs):
        return round(sorted(xs)[len(xs) // 2] / 1e3, 2)

    return {"windows": n, "steps": steps, "window_us": med(totals), "steps_us": [med(x) for x in per_step],
            "host_us": round(sum(med(x) for x in per_step), 1), "sync_tail_us": med(tails),
            "counters": {k: (med(v) if k.endswith("_ns") else sorted(v)[len(v) // 2]) for k, v in ctr.items() if v}}


def steady_block(R: Rank, res: dict, steps: int, dim: int) -> dict:
    st = res["stats"]
    el, total = res["el"], res["rows"]
    out = {
        "steps": steps,
        "timed_s": round(el, 6),
        "records_per_s": round(total / el, 1),
        "ms_per_step": round(el / steps * 1000, 4),
        "gb_per_s": round(total / el * dim * 4 / 1e9, 3),
        "ring_slots": res["occ"]["n_slots"],
        "prefilled_slots_at_t0": res["occ"]["prefilled"],
        "steps_per_ring": round(steps / max(1, res["occ"]["n_slots"]), 1),
        "vs_baseline": round(total / el / BASELINE_VALUE, 3),
        "commit_p50_us": round(st["commit_p50_us"], 2),
        "commit_p99_us": round(st["commit_p99_us"], 2),
        "commit_latency_p50_us": round(st["commit_latency_p50_us"], 2),
        "commit_latency_p99_us": round(st["commit_latency_p99_us"], 2),
        "commits": st["commits"],
        "worker_fill_us_per_batch": round(st.get("worker_fill_us_per_batch", 0.0), 2),
        "verify_wait_us_per_batch": round(st.get("verify_wait_us_per_batch", 0.0), 3),
    }
    if st.get("mirror_copies"):
        # HBM mirror: segments read from the pinned log instead (buffer busy / copy still in flight)
        out["mirror"] = {k: st.get(k, 0) for k in ("mirror_copies", "mirror_fallbacks", "mirror_pending_fallbacks",
                                                   "mirror_backoffs", "split_launches")}
    if "cpu" in res:
        out["cpu"] = res["cpu"]
    if R.world > 1:
        out["per_rank_records_per_s"] = [round(r / e, 1) for e, r in res["per_rank"]]
        out["lockstep_agreements"] = st.get("lockstep_agreements", 0)
        out["lockstep_wait_us_per_step"] = round(st.get("lockstep_wait_us_per_batch", 0.0), 2)
        out["lockstep_step_wait_max_us"] = round(st.get("lockstep_step_wait_max_us", 0.0), 1)
    return out


def lockstep_trace_summary(recs) -> dict:
    """TORCHKAFKA_LOCKSTEP_TRACE=1: where an agreement's round trip went, host clock, µs (p50 / p90):
    issuing it, the steps delivered before it was needed (slack), waiting for it, issue to result."""
    recs = [r for r in recs if r[3] > 0]

    def q(xs):
        xs = sorted(xs)
        return [round(xs[int(len(xs) * f)] / 1e3, 1) for f in (0.5, 0.9)] if xs else None

    return {"agreements": len(recs), "issue_us": q([r[1] - r[0] for r in recs]),
            "slack_us": q([r[2] - r[1] for r in recs]), "wait_us": q([r[3] - r[2] for r in recs]),
            "round_trip_us": q([r[3] - r[0] for r in recs])}


def _bridge_counters(loader) -> dict:
    """Where the bridges' fetch threads spent their time, summed over partitions and threads."""
    keys = ("bytes", "wire_bytes", "recv_ns", "ingest_ns", "inflate_ns", "inflated_batches", "inflated_bytes")
    out = {k: 0 for k in keys}
    out["fetch_wait_ns"] = out["fetch_threads"] = out["inflate_threads"] = 0
    for br in loader._bridges:
        for st in br.stats():
            for k in keys:
                out[k] += int(st[k])
        out["fetch_wait_ns"] += int(br._r.fetch_wait_ns)
        out["fetch_threads"] += int(br._r.fetch_threads)
        out["inflate_threads"] += int(br._r.inflate_threads)
    return out


def bridge_codec_block(R: "Rank", args, broker, mine, n_parts, codec, steps, warm, make_loader, server, dtype,
                       live: bool = True) -> dict:
    """bridge_<codec> (VERDICT r4 "do this" 6): the same records served as compressed RecordBatches.

    Setup (untimed): this rank's partitions of the topic are compressed batch by batch, as a
    producer with ``compression_type=codec`` writes them, into a staging topic; the served topic
    gets the warm-up's share.  The rest is appended to the served topic when the timed steps start
    (a live topic whose producer runs ahead), so every timed batch was fetched, inflated by a
    bridge fetch thread straight into the replica log (codecs.h ``decompress_into``) and then
    CRC-checked and decoded on the device inside the timed region.  ``live=False``: the whole topic
    is produced before the timed steps (the bridge and the decode alone, without the producer).
    ``producer``: when the producer's appends ended, against the timed region -- a producer still
    appending at the end of the timed steps is what the bridge waited for (fetch_wait)."""
    B = args.batch_size
    tag = codec if live else f"{codec}_static"
    stage, topic = f"stage_{tag}", f"bench_{tag}"
    broker.create_topic(stage, n_parts)
    broker.create_topic(topic, n_parts)
    per = int(math.ceil((warm + steps) * B * 1.1 / len(mine))) + B
    warm_per = int(math.ceil(warm * B * 1.5 / len(mine))) + B
    t = time.perf_counter()
    packed = broker.copy_compressed("bench", stage, codec, partitions=mine, max_records=per)
    compress_s = time.perf_counter() - t
    broker.copy_compressed(stage, topic, None, partitions=mine, max_records=warm_per if live else per)
    ld = make_loader(f"bench-bridge-{tag}", dtype, args.h2d, servers=server, topic=topic)
    from torchkafka_amd import auto_commit

    bit = BlockGuard(iter(auto_commit(ld)), ld)
    try:
        return _bridge_codec_timed(R, args, ld, bit, codec, steps, warm, live, broker, stage, topic, mine, per,
                                   warm_per, packed, compress_s)
    finally:
        bit.close()
        ld.close()  # (also after a failure: a lockstep transport leaves, the other ranks stop at once)


def _bridge_codec_timed(R, args, ld, bit, codec, steps, warm, live, broker, stage, topic, mine, per, warm_per,
                        packed, compress_s) -> dict:
    for _ in range(warm):
        next(bit)
    c0 = _bridge_counters(ld)
    err = []
    prod = {}

    def produce():
        t = time.perf_counter()
        try:
            if live:
                info = broker.copy_compressed(stage, topic, None, partitions=mine, start_record=warm_per,
                                              max_records=per)
                prod.update(batches=info["batches"], bytes=info["compressed_bytes"])
        except Exception as e:  # noqa: BLE001 - reported below
            err.append(e)
        prod["start"], prod["end"] = t, time.perf_counter()

    pub = threading.Thread(target=produce, name=f"bench-produce-{codec}")
    t_pub = time.perf_counter()
    pub.start()
    try:
        res = time_steps(R, bit, steps, ld)
        t_end = time.perf_counter()
    finally:
        pub.join()  # (also when the block failed: the producer's appends end on their own)
    c1 = _bridge_counters(ld)
    if err:
        raise err[0]
    blk = steady_block(R, res, steps, args.dim)
    d = {k: c1[k] - c0[k] for k in c1 if k not in ("fetch_threads", "inflate_threads")}
    el = res["el"]
    thread_s = c1["fetch_threads"] * el
    # compressed partitions are inflated by an inflater thread per fetch thread (replicator.cpp),
    # overlapping the fetch thread's wait for its next Fetch response
    inflater_s = (c1["inflate_threads"] or c1["fetch_threads"]) * el
    inflate_s, recv_s, wait_s = d["inflate_ns"] / 1e9, d["recv_ns"] / 1e9, d["fetch_wait_ns"] / 1e9
    other_ingest_s = max(0.0, d["ingest_ns"] / 1e9 - inflate_s)
    blk.update({
        "compression": codec,
        "served_as": f"{codec} RecordBatches ({packed['batches']} batches of {args.records_per_batch} records per "
                     "rank), produced into the served topic as the timed steps start",
        "compression_ratio": round(packed["raw_bytes"] / max(1, packed["compressed_bytes"]), 2),
        "wire_gb_per_s": round(d["wire_bytes"] / el / 1e9, 3),
        "inflated_gb_per_s": round(d["inflated_bytes"] / el / 1e9, 3),
        "inflated_batches_in_timed_region": d["inflated_batches"],
        "fetch_threads": c1["fetch_threads"],
        "inflate_threads": c1["inflate_threads"],
        "inflate_gb_per_s_per_thread": round(d["inflated_bytes"] / max(1e-9, inflate_s) / 1e9, 3),
        # over the timed region: a fetch thread's share reading record sets off the socket and
        # waiting for Fetch responses; an inflater's share inflating (decode + fresh CRC) and in
        # the rest of the ingest walk (CRC of the compressed batch, index) -- the remainder of
        # each is flow control and idle
        "fetch_thread_time_share": {"recv": round(recv_s / thread_s, 3), "fetch_wait": round(wait_s / thread_s, 3)},
        "inflater_time_share": {"inflate": round(inflate_s / inflater_s, 3),
                                "other_ingest": round(other_ingest_s / inflater_s, 3)},
        "compress_setup_s": round(compress_s, 2),
        "producer": ({"appends_s": round(prod["end"] - prod["start"], 4),
                      "ended_before_timed_end_s": round(t_end - prod["end"], 4),
                      "gb_per_s": round(prod.get("bytes", 0) / max(1e-9, prod["end"] - prod["start"]) / 1e9, 3)}
                     if live else "the whole topic produced before the timed steps"),
        "bridge_errors": sum(br.errors for br in ld._bridges),
    })
    return blk


def record_bytes(args) -> int:
    """Log bytes of one synthetic record: the f32 values, the 8-byte key and the record framing
    (~20 B of varints), plus its share of the 61-byte RecordBatch header."""
    return args.dim * 4 + 8 + 24 + (61 + args.records_per_batch - 1) // args.records_per_batch


def memory_preflight(R: "Rank", need_per_rank: int) -> dict:
    """The backlog every local rank writes into /dev/shm (and later pins) against what the host has:
    free space of /dev/shm and MemAvailable, shared by the local ranks.  ``scale`` < 1 tells the
    caller how far to shorten the timed blocks so that 1.25x the need fits."""
    local = int(os.environ.get("LOCAL_WORLD_SIZE", R.world))
    out = {"bytes_per_rank": need_per_rank, "local_ranks": local}
    room = []
    try:
        st = os.statvfs("/dev/shm")
        out["shm_free"] = st.f_bavail * st.f_frsize
        room.append(out["shm_free"])
    except OSError:
        pass
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    out["mem_available"] = int(line.split()[1]) * 1024
                    room.append(out["mem_available"])
    except OSError:
        pass
    budget = min(room) / max(1, local) if room else float("inf")
    out["scale"] = 1.0 if need_per_rank * 1.25 <= budget else budget / (need_per_rank * 1.25)
    return out


def run_config_blocks(R: "Rank", args) -> dict:
    """BASELINE configs 4, 5 and 1 and the RCCL-lockstep steady state, each on a broker of its own
    (N = 1 only: these are single-GPU configurations)."""
    import importlib

    names = [b for b in args.config_blocks.split(",") if b]
    out: dict = {}
    if R.world != 1 or not names:
        return out
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "benchmarks")
    if here not in sys.path:
        sys.path.insert(0, here)
    dev = str(R.device)
    on_gpu = R.device.type == "cuda"
    for name in names:
        t0 = time.perf_counter()
        try:
            got = _config_block(R, args, m_import=importlib.import_module, name=name, dev=dev, on_gpu=on_gpu)
        except Exception as e:  # noqa: BLE001 - reported in the line, the run goes on
            out[name] = {"error": f"{type(e).__name__}: {e}"[:500], "block_wall_s": round(time.perf_counter() - t0, 2)}
            _progress(R, f"{name} block failed: {e}")
            continue
        if got is None:
            continue
        name, res = got
        res["block_wall_s"] = round(time.perf_counter() - t0, 2)
        _progress(R, f"{name} block done in {res['block_wall_s']} s")
        out[name] = res
    return out


def _config_block(R: "Rank", args, m_import, name: str, dev: str, on_gpu: bool):
    """One of run_config_blocks' blocks: (the name it is reported under, its result), or None."""
    if name == "compute" and on_gpu:
        m = m_import("compute_overlap")
        res = {}
        for wl, h2d in (("config2", "zerocopy"), ("config2", "dma"), ("config4", "auto")):
            a = m.parse(["--workload", wl, "--h2d", h2d, "--steps", str(args.compute_steps), "--device", dev,
                         "--verify", args.verify])
            res[f"{wl}_{h2d}"] = m.run(a, sync=R.sync)
        name = "steady_compute"
    elif name == "train" and on_gpu:
        m = m_import("train_step")
        res = {}
        for wl, h2d in (("config2", "zerocopy"), ("config2", "dma"), ("config4", "auto")):
            a = m.parse(["--workload", wl, "--h2d", h2d, "--steps", str(args.train_steps), "--device", dev,
                         "--verify", args.verify])
            res[f"{wl}_{h2d}"] = m.run(a, sync=R.sync)
        name = "train_step"
    elif name == "config4" and on_gpu:
        m = m_import("config4_json_varlen")
        a = m.parse(["--steps", str(args.config4_steps), "--device", dev, "--verify", args.verify])
        res = m.run(a, sync=R.sync)
        res.pop("loader", None)
    elif name == "config5" and on_gpu:
        m = m_import("config5_large_messages")
        a = m.parse(["--steps", str(args.config5_steps), "--device", dev, "--verify", args.verify])
        res = m.run(a, sync=R.sync)
        res.pop("loader", None)
    elif name == "process":
        m = m_import("process_override")
        res = m.run(m.parse(["--steps", str(args.process_steps), "--device", dev]), sync=R.sync)
        name = "process_override"
    elif name == "config1":
        m = m_import("config1_cpu_plumbing")
        res = m.run(m.parse(["--records", str(args.config1_records)]))
    else:
        return None
    return name, res


def run_rank(args) -> int:
    R = Rank(args)
    torch, dist = R.torch, R.dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, Key, auto_commit
    from torchkafka_amd.broker import SyntheticBroker
    from torchkafka_amd.parallel import shard_partitions
    from torchkafka_amd.utils.topology import bind_to_gpu_numa

    rank, world = R.rank, R.world
    if not args.device and not args.no_numa:
        # the broker log this rank fills, its ring and its workers all live on its GPU's socket
        bind_to_gpu_numa(R.local_rank)
    dtypes = {"bf16": torch.bfloat16, "fp8": torch.float8_e4m3fn, "f16": torch.float16, "f32": torch.float32}
    device = R.device
    # lockstep: the agreement every step runs before a batch is delivered and committed
    if args.lockstep == "off":
        lockstep = False
    elif args.lockstep == "auto":
        lockstep = True  # the loader's transport choice: shared memory when every rank is on this host
    else:
        lockstep = args.lockstep  # a forced transport agrees every step, also at N = 1

    class Records(KafkaDataset):
        schema = FixedWidth(torch.float32, (args.dim,))

    class Labelled(KafkaDataset):
        schema = FixedWidth(torch.float32, (args.dim,)) + Key()

    # --- broker: one per job (every rank of the job shares its launcher's pid and port)
    tag = f"{os.getppid()}-{os.environ.get('MASTER_PORT', '0')}" if world > 1 else f"{os.getpid()}"
    url = f"shm://tkbench-{tag}"
    n_parts = args.partitions_per_gpu * world
    B = args.batch_size
    broker = SyntheticBroker.create(url, log_capacity=1 << 34, index_capacity=1 << 22)
    broker.create_topic("bench", n_parts)
    # backlog per owned partition: every batch the timed loop and the warm-up consume, plus what the
    # workers prefetch into their ring slots, with headroom (the secondary blocks re-read it from the
    # earliest offset under consumer groups of their own)
    mine = shard_partitions(n_parts, rank, world)
    ring_guess = args.workers * (args.slots_per_worker or 8)
    # >= 0.25 s on the GPU; a CPU dry run keeps its backlog (host memory) small
    steady = (args.steady_steps if args.steady_steps is not None
              else max(50 * ring_guess, 50000) if device.type == "cuda" else 2000)
    extra = [b for b in args.extra_blocks.split(",") if b]
    if device.type != "cuda":
        extra = [b for b in extra if b not in ("dma", "rccl", "rccl_sync", "verify")]
    if args.same_device:  # several ranks on one GPU: RCCL needs a device per rank
        extra = [b for b in extra if b not in ("rccl", "rccl_sync")]
    extra_steps = args.extra_steps if args.extra_steps is not None else steady
    if extra_steps <= 0:
        extra = []
    extra_warm = max(50, args.warmup)

    bsteps = args.bridge_steps if args.bridge_steps is not None else (8000 if device.type == "cuda" else 20)

    def backlog(steady_n, extra_n):
        # every block re-reads the topic from the earliest offset under a group of its own: the
        # longest one sets the backlog (a block that outran it would wait for records forever)
        consumed = max(args.warmup + args.steps * (1 + args.window_trace) + steady_n,
                       (extra_warm + extra_n) if extra else 0, (extra_warm + bsteps) if bsteps > 0 else 0)
        batches = consumed + args.workers * ((args.slots_per_worker or 8) + 2)
        return int(math.ceil(batches * B * 1.25 / max(1, len(mine)))) + B

    per_part = backlog(steady, extra_steps)
    preflight = memory_preflight(R, per_part * len(mine) * record_bytes(args))
    if preflight["scale"] < 1.0:
        # not enough shared memory / RAM for every local rank's backlog: shorten the steady blocks
        steady = int(steady * preflight["scale"])
        extra_steps = int(extra_steps * preflight["scale"])
        per_part = backlog(steady, extra_steps)
        preflight["shrunk_to"] = {"steady_steps": steady, "extra_steps": extra_steps,
                                  "bytes_per_rank": per_part * len(mine) * record_bytes(args)}
        if steady < 2000:
            print(f"[bench] rank {rank}: not enough memory for the backlog ({preflight}): refusing", file=sys.stderr)
            return 2
    t_fill = time.perf_counter()
    broker.fill("bench", per_part, "fixed_f32", size=args.dim, partitions=mine,
                records_per_batch=args.records_per_batch, threads=min(16, len(mine)), keyed=True)
    t_fill = time.perf_counter() - t_fill

    R.init_group()

    def make_loader(group: str, dtype, h2d: str, servers: str = url, commit: str = "async", ds=Records,
                    verify: str | None = None, lockstep_mode=None, topic: str = "bench"):
        return DeviceLoader(
            ds.placeholder(), B, num_workers=args.workers, device=device, dtype=dtype,
            slots_per_worker=args.slots_per_worker, prefetch=args.prefetch, rank=rank, world_size=world,
            in_order=args.in_order, h2d=h2d, copy_streams=args.copy_streams,
            **({"lockstep_depth": args.lockstep_depth} if args.lockstep_depth is not None else {}),
            **({"lockstep_commit_every": args.lockstep_commit_every} if args.lockstep_commit_every is not None
               else {}),
            event_every=args.event_every, numa_bind=not args.no_numa,
            **({"coalesce": args.coalesce} if args.coalesce is not None else {}),
            **({"decode_streams": args.decode_streams} if args.decode_streams is not None else {}),
            coalesce_wait_us=args.coalesce_wait_us, decode=args.decode,
            lockstep=lockstep if lockstep_mode is None else lockstep_mode,
            mirror_chunk_mib=args.mirror_chunk_mib, commit=commit, verify=verify or args.verify,
            **({"lockstep_timeout": 120.0} if lockstep_mode == "rccl" and world > 1 else {}),
            **({"mirror_chunks": args.mirror_chunks} if args.mirror_chunks else {}),
            worker_init_fn=ds.init_worker(topic, bootstrap_servers=servers, group_id=group,
                                          auto_offset_reset="earliest", check_crcs=not args.no_crc),
        )

    def describe(loader) -> tuple[str, str]:
        h2d = loader.plan.resolve_h2d(loader._slot_capacity()) if device.type == "cuda" else "n/a (cpu)"
        decode = ("host workers" if not loader.plan.span else
                  "device (gfx950 CRC32C + decode from an HBM mirror filled by SDMA copies)"
                  if loader.plan.mirror else "device (gfx950 CRC32C + decode from pinned logs)")
        return h2d, decode

    loader = make_loader("bench", dtypes[args.dtype], args.h2d)
    it = iter(auto_commit(loader))
    x = next(it)  # forks workers, initialises HIP / the RCCL lockstep
    if device.type == "cuda":
        torch.cuda.set_device(device)
    ranks_check = R.check_ranks()
    lock_info = dict(loader.lockstep_info)

    for _ in range(max(0, args.warmup - 1)):
        x = next(it)
    head_trace = [] if args.window_trace > 0 else None
    head = time_steps(R, it, args.steps, loader, head_trace)
    if head_trace and rank == 0:
        print(json.dumps({"headline_trace_us": [round(x * 1e6, 1) for x in head_trace]}), file=sys.stderr)
    elapsed, total_rows, stats = head["el"], head["rows"], head["stats"]
    value = total_rows / elapsed
    h2d_desc, decode_desc = describe(loader)

    if args.window_trace > 0 and rank == 0:
        print(json.dumps({"window_trace": window_trace(R, it, args.steps, args.window_trace, loader)}), file=sys.stderr)

    # Steady state, same loader, right after the headline: many times the ring depth, so the batches
    # the workers had prefilled before t0 are a small part of it and the producer side (fetch, pack,
    # publish) is inside the timed region.
    steady_out = s_stats = None
    if steady > 0:
        sres = time_steps(R, it, steady, loader)
        s_stats = sres["stats"]
        steady_out = steady_block(R, sres, steady, args.dim)
        _progress(R, f"steady_state {steady_out['records_per_s']:.0f} rec/s")
        if args.stats and rank == 0:
            print(json.dumps({"ring_at_steady_t0": sres["occ"]}), file=sys.stderr)
        x = sres["last"]

    # check what landed on the device: the last batch's records must be this rank's partitions
    parts = set(int(p) for p in x.float()[:, 1].tolist())
    assert parts <= set(mine), f"rank {rank} received foreign partitions {parts - set(mine)}"
    it.close()  # normal end of the auto_commit generator: final commit + worker shutdown
    loader.close()
    if world > 1:
        R.barrier()
    committed = broker.committed_offsets("bench", "bench")

    # secondary blocks: fresh loaders (own consumer groups) over the same retained topic
    extra_out = {}
    other_verify = "commit" if args.verify == "deliver" else "deliver"

    def extra_block(name: str) -> None:
        """One secondary steady block: a fresh loader (its own consumer group) over the retained topic."""
        dt = torch.float32 if name == "f32" else dtypes[args.dtype]
        own_group = False
        rccl_block = name in ("rccl", "rccl_sync")
        shm_block = name in ("shm", "shm_sync")
        if (rccl_block or shm_block) and not dist.is_initialized() and os.environ.get("TK_BENCH_NO_TORCH_NCCL") != "1":
            # a world-1 nccl group; one all-reduce on it makes torch's own RCCL communicator and its
            # streams, as a DDP job's gradient all-reduce does at N > 1 -- the N = 8 queue layout,
            # rehearsed on one GPU (the loader's own transport carries every agreement)
            os.environ["MASTER_ADDR"] = "127.0.0.1"
            os.environ["MASTER_PORT"] = str(_free_port())
            on_gpu = device.type == "cuda"
            dist.init_process_group("nccl" if on_gpu else "gloo", rank=0, world_size=1)
            dist.all_reduce(torch.ones(1, device=device))
            if on_gpu:
                torch.cuda.synchronize(device)
                os.environ["TORCHKAFKA_TORCH_NCCL_ACTIVE"] = "1"
            own_group = True
        ld = make_loader(f"bench-{name}", dt, "dma" if name == "dma" else args.h2d,
                         ds=Labelled if name == "label" else Records,
                         verify=other_verify if name == "verify" else None,
                         commit="sync" if name in ("rccl_sync", "shm_sync") else "async",
                         lockstep_mode="rccl" if rccl_block else "shm" if shm_block else None)
        eit = BlockGuard(iter(auto_commit(ld)), ld)
        try:
            extra_timed(name, ld, eit, rccl_block, shm_block)
        finally:
            eit.close()
            ld.close()  # (a failed block: its lockstep transport leaves, the other ranks stop at once)
            if own_group:
                dist.destroy_process_group()
                os.environ.pop("TORCHKAFKA_TORCH_NCCL_ACTIVE", None)
        if world > 1:
            R.barrier()

    def extra_timed(name: str, ld, eit, rccl_block: bool, shm_block: bool) -> None:
        for _ in range(extra_warm):
            next(eit)
        if os.environ.get("TK_BENCH_TEST_FAIL_BLOCK") == name and rank == world - 1:
            # tests only: one rank's block fails after its warm-up, as a failing next() would
            eit.fail(RuntimeError(f"test failure injected into block {name} on rank {rank}"))
        eres = time_steps(R, eit, extra_steps, ld)
        if name == "label":  # (features, label): the label is the key the broker wrote, offset % 1000
            xv, lab = eres["last"]
            if lab.dtype != torch.int64 or lab.shape != (xv.shape[0],) or not bool(((lab >= 0) & (lab < 1000)).all()):
                raise RuntimeError(f"label column mismatch: {lab.dtype} {tuple(lab.shape)}")
        blk = steady_block(R, eres, extra_steps, args.dim)
        blk["dtype"] = "f32" if name == "f32" else args.dtype
        blk["h2d"], blk["decode"] = describe(ld)
        blk["verify"] = ld.verify
        key = f"steady_{name}"
        if rccl_block or shm_block:
            st = eres["stats"]
            blk["commit"] = ("sync (commit, then the agreement: a cross-rank barrier per step)"
                             if name.endswith("_sync") else "async (commits land at agreements)")
            blk["commits_per_step"] = round(st["commits"] / max(1, extra_steps), 4)
            blk["batches_per_commit"] = round(extra_steps / max(1, st["commits"]), 2)
            blk["lockstep"] = dict(ld.lockstep_info)
            blk["lockstep_agreements"] = st.get("lockstep_agreements", 0)
            blk["lockstep_wait_us_per_step"] = round(st.get("lockstep_wait_us_per_batch", 0.0), 3)
            blk["lockstep_issue_us_per_step"] = round(st.get("lockstep_issue_us_per_batch", 0.0), 3)
            blk["lockstep_step_wait_max_us"] = round(st.get("lockstep_step_wait_max_us", 0.0), 1)
            rc = getattr(getattr(ld, "_run", None), "rccl", None)
            if rc is not None and os.environ.get("TORCHKAFKA_LOCKSTEP_TRACE") == "1":
                blk["lockstep_trace"] = lockstep_trace_summary(rc.take_trace())
        if name == "verify":
            key = "steady_unverified" if ld.verify == "commit" else "steady_verified"
            blk["verify_wait_us_per_batch"] = round(eres["stats"].get("verify_wait_us_per_batch", 0.0), 3)
        extra_out[key] = blk
        _progress(R, f"{key} {blk['records_per_s']:.0f} rec/s")

    def guarded(key: str, out: dict, fn) -> None:
        """Runs one secondary block; a failure is reported in the line under ``key`` instead of ending
        the run (every rank of a lockstepped block fails with it: the failing rank's transport leaves)."""
        try:
            fn()
        except Exception as e:  # noqa: BLE001 - reported in the line
            out[key] = {"error": f"{type(e).__name__}: {e}"[:500]}
            _progress(R, f"{key} failed: {e}")
            if world > 1:
                R.barrier()

    # the RCCL blocks at N > 1 run last (after the bridge blocks): the first multi-GPU runs of the
    # native RCCL lockstep -- a failure there is reported in the line instead of ending the run
    late = [b for b in extra if world > 1 and b in ("rccl", "rccl_sync")]
    if os.environ.get("TK_BENCH_TEST_LATE_HANG") == "1" and world > 1:
        late.append("test_hang")  # tests only: a late block that never returns (the watchdog's path)
    for name in extra:
        if name not in late:
            guarded(f"steady_{name}", extra_out, lambda name=name: extra_block(name))

    # the Kafka-protocol route: this rank's partitions over a loopback wire server -> bridge replica
    bridge_out = None
    if bsteps > 0:
        from torchkafka_amd.broker import NativeWireServer

        srv = NativeWireServer(broker, profile="kafka4").start()
        bridge_out = {"server": "NativeWireServer (C++), loopback TCP, Kafka 4.x protocol profile",
                      "replica": "KafkaBridge ring replica of this rank's partitions (static shard)"}

        def bridge_mode(mode: str, steps: int) -> None:
            ld = make_loader(f"bench-bridge-{mode}", dtypes[args.dtype], args.h2d, servers=srv.address,
                             commit=mode)
            bit = BlockGuard(iter(auto_commit(ld)), ld)
            try:
                for _ in range(extra_warm):
                    next(bit)
                for br in ld._bridges:
                    br.take_forward_ns()
                bres = time_steps(R, bit, steps, ld)
                blk = steady_block(R, bres, steps, args.dim)
                rtt = sorted(x / 1e3 for br in ld._bridges for x in br.take_forward_ns())
                if mode == "async":
                    blk["commit_latency_means"] = "request of batch k+1 -> batch k stored in the replica's table"
                    blk["coordinator_rtt_p50_us"] = round(rtt[len(rtt) // 2], 1) if rtt else None
                    p99 = rtt[min(len(rtt) - 1, len(rtt) * 99 // 100)] if rtt else None
                    blk["coordinator_rtt_p99_us"] = round(p99, 1) if rtt else None
                    blk["coordinator_commits"] = len(rtt)
                    blk["forward_interval_ms"] = 5
                else:
                    st = bres["stats"]
                    blk["commit_latency_means"] = ("request of batch k+1 -> batch k's OffsetCommit answered by "
                                                   "the coordinator (sync_commit_*)")
                    blk["sync_commit_p50_us"] = round(st["sync_commit_p50_us"], 1)
                    blk["sync_commit_p99_us"] = round(st["sync_commit_p99_us"], 1)
                    blk["sync_commits"] = st["sync_commits"]
                blk["bridge_errors"] = sum(br.errors for br in ld._bridges)
                bridge_out[mode] = blk
                _progress(R, f"bridge {mode} {blk['records_per_s']:.0f} rec/s")
            finally:
                bit.close()
                ld.close()
            if world > 1:
                R.barrier()

        def bridge_codec(codec: str) -> None:
            static = codec.endswith("_static")
            name = codec[:-len("_static")] if static else codec
            bridge_out[codec] = bridge_codec_block(R, args, broker, mine, n_parts, name, bsteps, extra_warm,
                                                   make_loader, srv.address, dtypes[args.dtype], live=not static)
            _progress(R, f"bridge {codec} {bridge_out[codec]['records_per_s']:.0f} rec/s")
            if world > 1:
                R.barrier()

        try:
            for mode, steps in (("async", bsteps), ("sync", max(1, bsteps // 4))):
                guarded(mode, bridge_out, lambda mode=mode, steps=steps: bridge_mode(mode, steps))
            for codec in [c for c in args.bridge_codecs.split(",") if c]:
                guarded(codec, bridge_out, lambda codec=codec: bridge_codec(codec))
        finally:
            srv.close()

    config_out = run_config_blocks(R, args)

    def make_out() -> dict:
        return {
            "metric": BASELINE_METRIC,
            "value": round(value, 1),
            "unit": "records/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_VALUE, 3),
            "dtype": args.dtype,
            "data": ("synthetic (Kafka RecordBatch v2 records in the shared-memory broker, "
                     "random-free deterministic f32)"),
            "config": {
                "model": (f"KafkaDataset FixedWidth f32[{args.dim}] ({args.dim * 4} B records) -> {args.dtype} "
                          "via gfx950 collate"),
                "global_batch": B * world,
                "seq_len": args.dim,
                "parallelism": f"dp{world}",
                "partitions": n_parts,
                "num_workers": args.workers,
                "verify": ("deliver (a batch is handed out after its device CRC32C verdict)" if args.verify == "deliver"
                           else "commit (the CRC32C verdict gates the commit only)"),
                "commit": (f"auto_commit: {(s_stats or stats)['commits']} commits in "
                           f"{steady if s_stats else args.steps} steps "
                           f"({(steady if s_stats else args.steps) / max(1, (s_stats or stats)['commits']):.2f} "
                           "batches per commit)") + (
                    "" if not lock_info else ", RCCL lockstep" if lock_info.get("transport") == "rccl"
                    else ", node-local shared-memory lockstep" if lock_info.get("transport") == "shm"
                    else f", lockstep ({lock_info.get('backend', 'host')} all-reduce)"),
                "h2d": h2d_desc,
                "decode": decode_desc,
                "bytes_per_step_per_gpu": B * args.dim * 4,
                "gb_per_s": round(value * args.dim * 4 / 1e9, 3),
                "commit_p99_us": round(stats["commit_p99_us"], 2),
            },
            "launcher": os.environ.get("TK_BENCH_LAUNCHER", "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                       else "single process"),
            "ranks": ranks_check,
            "lockstep": lock_info or None,
            "rccl_nranks": lock_info.get("rccl_nranks"),
            "per_rank_records_per_s": [round(r / e, 1) for e, r in head["per_rank"]],
            # request of batch k+1 -> batch k's offsets stored, incl. the lockstep agreement and the
            # wait for batch k's on-device CRC verdict (steady-state block when it ran)
            "commit_latency_p50_us": round((s_stats or stats)["commit_latency_p50_us"], 2),
            "commit_latency_p99_us": round((s_stats or stats)["commit_latency_p99_us"], 2),
            "timed_region_s": round(elapsed, 6),
            "prefilled_slots_at_t0": head["occ"]["prefilled"],
            "ring_slots": head["occ"]["n_slots"],
            "fill_s": round(t_fill, 2),
            "steady_state": steady_out,
            **extra_out,
            "bridge": bridge_out,
            **config_out,
            "memory_preflight": preflight,
            # the native binaries that ran, with the source sha compiled into each (ops.build_info)
            "native_build": _native_build(),
        }

    # The RCCL blocks at N > 1 run last, under a watchdog: the first multi-GPU runs of the native
    # RCCL lockstep must not cost the job its line.  A block that fails is reported in the line; if
    # they have not finished by the deadline (a hang in RCCL itself), every rank's watchdog puts the
    # line out without them (rank 0) and leaves.
    printed = threading.Lock()
    emitted = []

    def emit() -> None:
        with printed:
            if rank == 0 and not emitted:
                print(json.dumps(make_out()), flush=True)
            emitted.append(1)

    late_done = threading.Event()
    if late:
        late_s = float(os.environ.get("TK_BENCH_LATE_TIMEOUT", "300"))

        def watchdog() -> None:
            if late_done.wait(late_s):
                return
            for name in late:
                extra_out.setdefault(f"steady_{name}", {"error": f"did not finish within {late_s:.0f} s (watchdog)"})
            _progress(R, f"RCCL blocks did not finish within {late_s:.0f} s: the line goes out without them")
            emit()
            if rank == 0:
                broker.destroy()
            sys.stdout.flush()
            os._exit(0)

        threading.Thread(target=watchdog, daemon=True, name="bench-late-watchdog").start()
    for name in late:
        if name == "test_hang":
            time.sleep(3600)
        guarded(f"steady_{name}", extra_out, lambda name=name: extra_block(name))

    if rank == 0 and args.stats:
        print(json.dumps({"loader_stats": stats, "fill_s": t_fill,
                          "committed_sample": dict(list(committed.items())[:4])}),
              file=sys.stderr)
    emit()
    if world > 1:
        R.barrier()  # still under the watchdog: a rank stuck in RCCL must not hold the others here
        dist.destroy_process_group()
    late_done.set()
    if rank == 0:
        broker.destroy()
    return 0


def _native_build() -> dict:
    from torchkafka_amd.ops import build_info

    return {name: {"sha16": b["built_from"][:16] if b["built_from"] else None, "matches_tree": b["matches_tree"]}
            for name, b in build_info().items()}


def _progress(R, what: str) -> None:
    """One stderr line per finished block (rank 0): a long run shows where it is."""
    if R.rank == 0:
        print(f"[bench] {what} ({time.strftime('%H:%M:%S')})", file=sys.stderr, flush=True)


def main() -> int:
    args = parse()
    if os.environ.get("TK_BENCH_WATCHDOG"):
        # diagnostic: every N seconds, every thread's Python stack to stderr (a run that stalls)
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["TK_BENCH_WATCHDOG"]), repeat=True)
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.self_launch):
        return launch_ranks(args)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
