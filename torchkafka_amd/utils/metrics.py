"""Loader metrics: the reference has no timers or counters at all.

Cheap per-batch accounting kept on the hot path (a few integer adds):
records/bytes delivered, host time spent waiting for a ring slot vs issuing
the copy+collate, and commit latency samples for p50/p99 reporting.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field


def percentile(samples, q: float) -> float:
    if not samples:
        return float("nan")
    s = sorted(samples)
    k = (len(s) - 1) * q / 100.0
    lo = int(k)
    hi = min(lo + 1, len(s) - 1)
    return s[lo] + (s[hi] - s[lo]) * (k - lo)


@dataclass
class LoaderStats:
    batches: int = 0
    records: int = 0
    payload_bytes: int = 0
    wait_ns: int = 0
    issue_ns: int = 0
    commits: int = 0
    commit_failures: int = 0
    commit_ns: list = field(default_factory=list)
    # request of batch k+1 -> batch k's offsets stored (incl. lockstep / decode verdict / fence waits)
    commit_latency_ns: list = field(default_factory=list)
    # commit='sync': the wait for batch k's verdict + store + coordinator answer before batch k+1
    sync_commit_ns: list = field(default_factory=list)
    worker_fill_ns: int = 0
    worker_fills: int = 0
    ready_age_ns: int = 0
    worker_idle_ns: int = 0
    worker_slot_wait_ns: int = 0
    phase_commit_ns: int = 0   # native step driver: finish + commit of the previous batch
    phase_next_ns: int = 0     # native step driver: slot release/acquire (+H2D issue)
    phase_launch_ns: int = 0   # native step driver: collate launch (+event)
    phase_steps: int = 0
    events: int = 0            # completion events recorded (batched: fewer than batches)
    groups: int = 0            # coalesced launches (several batches collated by one kernel)
    coalesce_wait_ns: int = 0  # main thread waiting for a full group while the GPU was busy
    ahead_ns: int = 0  # main thread forming and launching device-decode groups ahead of delivery
    json_width_wait_ns: int = 0  # main thread waiting for a parse kernel to report a batch width
    occ_handed: int = 0        # slots launched on the GPU and not yet released, summed per step
    occ_staged: int = 0        # slots taken from the ring and not yet launched, summed per step
    occ_samples: int = 0
    release_ns: int = 0        # native next phase: slot releases (event queries + ring hand-back)
    poll_ns: int = 0           # native next phase: non-blocking stagings of READY slots
    polled: int = 0
    log_bytes_registered: int = 0  # h2d="direct": broker log bytes pinned in place so far
    log_bytes_unpinned: int = 0    # replica logs: consumed ranges unpinned again (kReleaseConsumed)
    log_register_ns: int = 0
    log_register_wait_ns: int = 0  # the launch thread waiting for the pin thread (growing logs)
    mirror_pending_fallbacks: int = 0  # mirror segments read from the pinned log: their copy was in flight
    mirror_bytes: int = 0     # h2d="dma" device decode: log bytes copied into the HBM mirror (SDMA)
    mirror_copies: int = 0
    split_launches: int = 0    # decode launches with each segment split over workgroups (HBM)
    mirror_fallbacks: int = 0  # segments read from the pinned log instead (buffer busy)
    mirror_backoffs: int = 0   # times the mirror stopped copying: its copies fell behind (log_mirror.h)
    lockstep_agreements: int = 0      # cross-rank agreements (collectives) issued
    lockstep_wait_ns: int = 0         # host time waiting for agreement results
    lockstep_issue_ns: int = 0        # host time issuing agreements (the transport's enqueue)
    verify_wait_ns: int = 0           # verify='deliver': host time waiting for a batch's device verdict
    lockstep_step_wait_max_ns: int = 0  # the most one delivered step waited for them
    started: float = field(default_factory=time.perf_counter)
    max_commit_samples: int = 100000

    def record_batch(self, rows: int, nbytes: int, wait_ns: int, issue_ns: int) -> None:
        self.batches += 1
        self.records += rows
        self.payload_bytes += nbytes
        self.wait_ns += wait_ns
        self.issue_ns += issue_ns

    def record_commit(self, ns: int) -> None:
        self.commits += 1
        if len(self.commit_ns) < self.max_commit_samples:
            self.commit_ns.append(ns)

    def record_sync_commit(self, ns: int) -> None:
        if len(self.sync_commit_ns) < self.max_commit_samples:
            self.sync_commit_ns.append(ns)

    def record_commit_latency(self, ns: int) -> None:
        if len(self.commit_latency_ns) < self.max_commit_samples:
            self.commit_latency_ns.append(ns)

    def reset(self) -> None:
        self.__init__()

    def summary(self) -> dict:
        el = time.perf_counter() - self.started
        c_us = [x / 1e3 for x in self.commit_ns]
        lat_us = [x / 1e3 for x in self.commit_latency_ns]
        return {
            "batches": self.batches,
            "records": self.records,
            "bytes": self.payload_bytes,
            "elapsed_s": el,
            "records_per_s": self.records / el if el > 0 else float("nan"),
            "host_wait_us_per_batch": self.wait_ns / 1e3 / max(self.batches, 1),
            "host_issue_us_per_batch": self.issue_ns / 1e3 / max(self.batches, 1),
            "worker_fill_us_per_batch": self.worker_fill_ns / 1e3 / max(self.worker_fills, 1),
            "ready_age_us_per_batch": self.ready_age_ns / 1e3 / max(self.worker_fills, 1),
            "worker_idle_us_per_batch": self.worker_idle_ns / 1e3 / max(self.worker_fills, 1),
            "worker_slot_wait_us_per_batch": self.worker_slot_wait_ns / 1e3 / max(self.worker_fills, 1),
            "native_commit_us_per_step": self.phase_commit_ns / 1e3 / max(self.phase_steps, 1),
            "native_next_us_per_step": self.phase_next_ns / 1e3 / max(self.phase_steps, 1),
            "native_launch_us_per_step": self.phase_launch_ns / 1e3 / max(self.phase_steps, 1),
            "events_per_batch": self.events / max(self.batches, 1),
            "group_launches_per_batch": self.groups / max(self.batches, 1),
            "coalesce_wait_us_per_batch": self.coalesce_wait_ns / 1e3 / max(self.batches, 1),
            "ahead_launch_us_per_batch": self.ahead_ns / 1e3 / max(self.batches, 1),
            "json_width_wait_us_per_batch": self.json_width_wait_ns / 1e3 / max(self.batches, 1),
            "slots_on_gpu_avg": self.occ_handed / max(self.occ_samples, 1),
            "slots_staged_avg": self.occ_staged / max(self.occ_samples, 1),
            "native_release_us_per_step": self.release_ns / 1e3 / max(self.phase_steps, 1),
            "native_poll_us_per_step": self.poll_ns / 1e3 / max(self.phase_steps, 1),
            "native_poll_us_per_slot": self.poll_ns / 1e3 / max(self.polled, 1),
            "log_mib_pinned": self.log_bytes_registered / 2**20,
            "log_mib_unpinned": self.log_bytes_unpinned / 2**20,
            "log_pin_ms": self.log_register_ns / 1e6,
            "log_pin_wait_ms": self.log_register_wait_ns / 1e6,
            "mirror_mib_copied": self.mirror_bytes / 2**20,
            "mirror_copies": self.mirror_copies,
            "split_launches": self.split_launches,
            "mirror_fallbacks": self.mirror_fallbacks,
            "mirror_pending_fallbacks": self.mirror_pending_fallbacks,
            "mirror_backoffs": self.mirror_backoffs,
            "lockstep_agreements": self.lockstep_agreements,
            "lockstep_wait_us_per_batch": self.lockstep_wait_ns / 1e3 / max(self.batches, 1),
            "lockstep_issue_us_per_batch": self.lockstep_issue_ns / 1e3 / max(self.batches, 1),
            "verify_wait_us_per_batch": self.verify_wait_ns / 1e3 / max(self.batches, 1),
            "lockstep_step_wait_max_us": self.lockstep_step_wait_max_ns / 1e3,
            "commits": self.commits,
            "commit_failures": self.commit_failures,
            "commit_p50_us": percentile(c_us, 50),
            "commit_p99_us": percentile(c_us, 99),
            "commit_latency_p50_us": percentile(lat_us, 50),
            "commit_latency_p99_us": percentile(lat_us, 99),
            "commit_latency_max_us": max(lat_us) if lat_us else float("nan"),
            "commit_latency_samples": len(lat_us),
            "sync_commit_p50_us": percentile([x / 1e3 for x in self.sync_commit_ns], 50),
            "sync_commit_p99_us": percentile([x / 1e3 for x in self.sync_commit_ns], 99),
            "sync_commits": len(self.sync_commit_ns),
        }


class StageTimer:
    """Named wall-clock stage accumulator (``with timer('h2d'): ...``)."""

    def __init__(self):
        self.totals: dict[str, float] = {}
        self.counts: dict[str, int] = {}

    def __call__(self, name: str):
        timer = self

        class _Ctx:
            def __enter__(self):
                self.t = time.perf_counter()

            def __exit__(self, *exc):
                timer.totals[name] = timer.totals.get(name, 0.0) + time.perf_counter() - self.t
                timer.counts[name] = timer.counts.get(name, 0) + 1

        return _Ctx()

    def report(self) -> dict:
        return {k: {"total_s": v, "count": self.counts[k], "mean_us": v / self.counts[k] * 1e6}
                for k, v in self.totals.items()}
