"""DeviceLoader's commit side: exact per-batch commits, sync commits, checkpoint / resume.

Every batch carries the exact offsets of the records packed in it, so a commit covers exactly
what the user finished (reference D3: kafka-python commits its position, prefetched records
included).  The commit of batch k happens when batch k+1 is requested, as the reference's
``auto_commit`` does (/root/reference/src/auto_commit.py:55-58); ``commit='sync'`` additionally
waits for the coordinator (and, under a cross-rank lockstep, makes the commit a per-step barrier)
before batch k+1 is handed out (/root/reference/src/kafka_dataset.py:130).  The committed offsets
are the checkpoint: :meth:`LoaderCommits.state_dict` / ``load_state_dict``.  Log
messages and levels are the reference's (kafka_dataset.py:124-143).
"""
from __future__ import annotations

import logging
import time

import torch

from ..client.errors import COMMIT_FAILED_ERRORS, CorruptRecordException, KafkaError
from ..ops.collate import _stream_ptr

_ds_logger = logging.getLogger("torchkafka.kafka_dataset")


class LoaderCommits:
    """Mixin of :class:`~torchkafka_amd.loader.DeviceLoader`: ``_pending_wms`` (finished,
    uncommitted watermark lists), ``_committed``, ``stats``, the live ``_run``."""

    def _finish_marker(self, wms):
        """Marks a batch finished; in ``commit_on='device'`` mode fenced by the user's queued GPU work."""
        t = time.perf_counter_ns()  # the user asked for the next batch: commit latency starts
        if self.commit_on == "device" and self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            return (wms, ev, t)
        return (wms, None, t)

    def _sync_commit(self, drv, debug: bool) -> int:
        """``commit='sync'``: every finished batch's verdict, local store and -- through the
        bridges -- the coordinator's OffsetCommit answer, before the next batch is handed out.
        Returns the commit status the next lockstep agreement carries to every rank: 2 stored,
        1 a CommitFailedError was logged and swallowed (the reference's kafka_dataset.py:131-135)."""
        t0 = time.perf_counter_ns()
        drv.drain_fenced(True)
        ok = self._commit_native(drv, debug)
        run = self._run
        if run is not None and run.table is not None:
            run.wait_worker_commits(30.0)  # each worker's consumer committed (and, bridged, forwarded)
        ok = self._sync_bridges(t0) and ok
        return 2 if ok else 1

    def _commit_logged(self, drv) -> None:
        """One native commit bracketed by the reference's DEBUG messages (kafka_dataset.py:124-143).

        With DEBUG enabled the native loops hand the commit back to Python (the step call is made
        with its inline commit off), so "Committing offsets." precedes the store as it does in the
        reference; without DEBUG the commit stays inside the one native step call.  With
        ``commit_sink='worker'`` the workers commit and log ("Committing offsets on worker %d."), as
        the reference's workers do, and the main process stays silent."""
        if self._sink == "worker":
            return self._log_commit(drv.commit_pending(), False)
        _ds_logger.debug("Committing offsets.")
        return self._log_commit(drv.commit_pending(), True)

    def _commit_native(self, drv, debug: bool) -> bool:
        if debug:
            return self._commit_logged(drv)
        return self._log_commit(drv.commit_pending(), False)

    def _log_commit(self, status: int, debug: bool) -> bool:
        """False when the commit failed (CommitFailedError: logged, swallowed)."""
        if status == -2:  # a device-parsed batch was malformed: it (and what follows) stays uncommitted
            raise CorruptRecordException(self._run.driver.parse_error())
        if status == -1:
            _ds_logger.error("Commit failed.")
            return False
        if status == 1 and debug:
            _ds_logger.debug("Committed offsets.")
        return True

    def _absorb_driver_stats(self, drv) -> None:
        st = drv.stats()
        self.stats.worker_fill_ns += st["fill_ns"]
        self.stats.worker_fills += st["fills"]
        self.stats.wait_ns += st["blocked_ns"]
        self.stats.ready_age_ns += st["ready_age_ns"]
        self.stats.worker_idle_ns += st.get("worker_idle_ns", 0)
        self.stats.worker_slot_wait_ns += st.get("worker_slot_wait_ns", 0)
        self.stats.phase_commit_ns += st["phase_commit_ns"]
        self.stats.phase_next_ns += st["phase_next_ns"]
        self.stats.phase_launch_ns += st["phase_launch_ns"]
        self.stats.phase_steps += st["phase_steps"]
        self.stats.events += st["events"]
        self.stats.batches += st.get("fast_batches", 0)
        self.stats.records += st.get("fast_records", 0)
        self.stats.issue_ns += st.get("fast_ns", 0)
        self.stats.groups += st.get("groups", 0)
        self.stats.coalesce_wait_ns += st.get("coalesce_wait_ns", 0)
        self.stats.ahead_ns += st.get("ahead_ns", 0)
        self.stats.json_width_wait_ns += st.get("json_width_wait_ns", 0)
        self.stats.occ_handed += st.get("occ_handed", 0)
        self.stats.occ_staged += st.get("occ_staged", 0)
        self.stats.occ_samples += st.get("occ_samples", 0)
        self.stats.release_ns += st.get("release_ns", 0)
        self.stats.poll_ns += st.get("poll_ns", 0)
        self.stats.polled += st.get("polled", 0)
        self.stats.log_bytes_registered = st.get("log_bytes_registered", 0)
        self.stats.log_bytes_unpinned = st.get("log_bytes_unpinned", 0)
        self.stats.log_register_ns = st.get("log_register_ns", 0)
        self.stats.log_register_wait_ns = st.get("log_register_wait_ns", 0)
        self.stats.mirror_bytes += st.get("mirror_bytes_copied", 0)
        self.stats.mirror_copies += st.get("mirror_copies", 0)
        self.stats.split_launches += st.get("split_launches", 0)
        self.stats.mirror_fallbacks += st.get("mirror_fallbacks", 0)
        self.stats.mirror_pending_fallbacks += st.get("mirror_pending_fallbacks", 0)
        self.stats.mirror_backoffs += st.get("mirror_backoffs", 0)
        self.stats.verify_wait_ns += st.get("verify_wait_ns", 0)
        self.stats.lockstep_agreements += st.get("lockstep_agreements", 0)
        self.stats.lockstep_wait_ns += st.get("lockstep_wait_ns", 0)
        self.stats.lockstep_issue_ns += st.get("lockstep_issue_ns", 0)
        self.stats.lockstep_step_wait_max_ns = max(self.stats.lockstep_step_wait_max_ns,
                                                   st.get("lockstep_step_wait_max_ns", 0))
        self.stats.commits += st["commits"]
        self.stats.commit_failures += st["commit_failures"]
        self.stats.commit_ns.extend(st["commit_ns"])
        self.stats.commit_latency_ns.extend(st.get("commit_latency_ns", ()))
        self._committed.update(dict(drv.committed()))
        drv.reset_stats()

    def _broker(self):
        from ..broker.synthetic import open_broker, resolve_url

        return open_broker(resolve_url(self._servers))

    def _sync_commit_py(self) -> int:
        """commit='sync' on the Python path: every finished batch stored (fences waited for) and,
        through the bridges / the workers' consumers, answered by the coordinator.  Returns the
        commit status for the lockstep (2 stored, 1 a CommitFailedError logged and swallowed)."""
        t0 = time.perf_counter_ns()
        failures = self.stats.commit_failures
        self._commit_finished(wait=True)
        run = self._run
        if run is not None and run.table is not None:
            run.wait_worker_commits(30.0)
        ok = self._sync_bridges(t0) and self.stats.commit_failures == failures
        return 2 if ok else 1

    def _commit_finished(self, wait: bool = False) -> None:
        """Commits the watermarks of every batch the user finished (exactly those)."""
        pending = self._pending_wms
        if not pending:
            return
        offsets: dict[int, int] = {}
        keep = []
        started = []
        for i, entry in enumerate(pending):
            wms, ev = (entry[0], entry[1]) if isinstance(entry, tuple) else (entry, None)
            if ev is not None and not wait and not ev.query():
                # in order: a later batch is never committed before an earlier one (the committed
                # offset must not go backwards when the earlier one completes)
                keep.extend(pending[i:])
                break
            if ev is not None and wait:
                ev.synchronize()
            if isinstance(entry, tuple) and len(entry) > 2:
                started.append(entry[2])
            for pidx, _first, nxt, _cnt in wms:
                if nxt > offsets.get(pidx, -1):
                    offsets[pidx] = nxt
        self._pending_wms[:] = keep
        if offsets:
            if self._commit(offsets):
                now = time.perf_counter_ns()
                for t in started:
                    self.stats.record_commit_latency(now - t)

    def _commit(self, offsets: dict[int, int]) -> bool:
        if self._sink == "worker":
            run = self._run
            if run is None or run.table is None or run.closed:
                raise RuntimeError("DeviceLoader commit_sink='worker': commit() must be called while iterating")
            t0 = time.perf_counter_ns()
            by_worker: dict[int, dict[int, int]] = {}
            for p, o in offsets.items():
                by_worker.setdefault(run.pidx_worker[p], {})[p] = o
            for w, offs in by_worker.items():
                run.table.publish(w, offs)  # that worker's consumer commits (and logs) them
            self._committed.update(offsets)
            self.stats.record_commit(time.perf_counter_ns() - t0)
            return True
        if self._group_id is None:
            raise RuntimeError("DeviceLoader cannot commit: no group_id (pass it to init_worker or DeviceLoader)")
        t0 = time.perf_counter_ns()
        b = self._broker().native
        g = b.group_index(self._group_id, True)
        _ds_logger.debug("Committing offsets.")
        ok = False
        try:
            b.commit(g, -1, 0, 0, [(p, int(o), "") for p, o in offsets.items()])
        except COMMIT_FAILED_ERRORS:
            _ds_logger.error("Commit failed.")
            self.stats.commit_failures += 1
        else:
            _ds_logger.debug("Committed offsets.")
            self._committed.update(offsets)
            ok = True
        self.stats.record_commit(time.perf_counter_ns() - t0)
        return ok

    def commit(self) -> None:
        """Commits every batch yielded so far (manual mode)."""
        run = self._run
        if run is not None and run.driver is not None and not run.closed:
            run.driver.finish_delivered(_stream_ptr(self.device))
            run.driver.drain_fenced(True)
            self._commit_logged(run.driver)
            self._absorb_driver_stats(run.driver)
        self._commit_finished(wait=True)

    def committed_offsets(self) -> dict[int, int]:
        """{partition index: committed offset} of every partition this loader committed (live during
        iteration: the native driver's commits are included)."""
        run = self._run
        if run is not None and run.driver is not None and not run.closed:
            self._committed.update(dict(run.driver.committed()))
        return dict(self._committed)

    def _absorb_delivered(self, drv) -> None:
        """The native driver's delivered positions, kept past its iteration."""
        pos = self._delivered_pos
        for pidx, nxt in drv.delivered_positions():
            if nxt > pos.get(pidx, -1):
                pos[pidx] = nxt

    def delivered_positions(self) -> dict[int, int]:
        """{partition index: position after every batch handed out so far} -- live during
        iteration; includes the checkpoint this loader resumed from."""
        run = self._run
        if run is not None and run.driver is not None and not run.closed:
            self._absorb_delivered(run.driver)
        return dict(self._delivered_pos)

    def state_dict(self, global_step: bool = False, group=None) -> dict:
        """Positions for a model checkpoint (the committed offsets ARE the checkpoint).

        ``global_step=False``: this rank's committed positions,
        ``{"version": 1, "group_id": g, "offsets": {topic: {partition: offset}}}``.

        ``global_step=True`` (DDP): every rank's positions at the END OF THE SAME STEP -- call it
        on every rank at the same step of the training loop (a collective).  Each rank contributes
        the positions after the batches it has handed out (not its committed table: under the
        async lockstep commits land at agreements, dozens of steps apart), one all-gather over
        ``group`` (a gloo group is made from the default group if it is not one) merges them, and
        the ranks' step counts must agree.  ``{"version": 2, "group_id", "global_step": S,
        "world_size": W, "offsets": {...every rank's partitions...}}``, identical on every rank;
        ``load_state_dict`` resumes from it on any number of ranks.  JSON-serialisable."""
        b = self._broker()
        if not global_step:
            offsets: dict[str, dict[int, int]] = {}
            for pidx, off in sorted(self.committed_offsets().items()):
                tp = b.tp_of(pidx)
                offsets.setdefault(tp.topic, {})[tp.partition] = int(off)
            return {"version": 1, "group_id": self._group_id, "offsets": offsets}
        import torch.distributed as dist

        pos = self.delivered_positions()
        step = self._global_step_base + self._steps_delivered
        world = 1
        merged = dict(pos)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            world = dist.get_world_size(group)
            grp = group if group is not None and dist.get_backend(group) == "gloo" else self._cpu_group(group)
            gathered: list = [None] * world
            dist.all_gather_object(gathered, (step, pos), group=grp)
            steps = sorted({g[0] for g in gathered})
            if len(steps) != 1:
                raise RuntimeError(f"state_dict(global_step=True): the ranks stand at different steps {steps}; call "
                                   "it on every rank at the same step of the loop")
            for _, p in gathered:
                for pidx, nxt in p.items():
                    if nxt > merged.get(pidx, -1):
                        merged[pidx] = nxt
        offsets = {}
        for pidx, off in sorted(merged.items()):
            tp = b.tp_of(pidx)
            offsets.setdefault(tp.topic, {})[tp.partition] = int(off)
        return {"version": 2, "group_id": self._group_id, "global_step": int(step), "world_size": world,
                "offsets": offsets}

    def _cpu_group(self, group=None):
        """A gloo group over the ranks of ``group``: ``group`` itself when it is gloo, else one made
        per distinct rank list (torch's new_group: a collective of EVERY rank of the job, members or
        not) and kept for the next call with the same ranks."""
        import torch.distributed as dist

        if dist.get_backend(group) == "gloo":
            return group
        ranks = tuple(range(dist.get_world_size())) if group is None else tuple(dist.get_process_group_ranks(group))
        cache = self.__dict__.setdefault("_gloo_groups", {})
        if ranks not in cache:
            cache[ranks] = dist.new_group(ranks=list(ranks), backend="gloo")
        return cache[ranks]

    def load_state_dict(self, state: dict) -> None:
        """Resumes from a checkpoint's offsets: they are committed for the group (an administrative
        commit, as ``kafka-consumer-groups --reset-offsets`` does), so the next iteration's workers
        start exactly there, like consumers restarting after a crash.  Call before iterating."""
        from ..client.records import TopicPartition

        if self._run is not None and not self._run.closed:
            raise RuntimeError("load_state_dict() must be called before iterating the loader")
        if int(state.get("version", 1)) not in (1, 2):
            raise ValueError(f"unsupported DeviceLoader state version {state.get('version')}")
        group = state.get("group_id") or self._group_id
        if group is None:
            raise RuntimeError("load_state_dict needs a group_id (in the state or the loader)")
        offs = {TopicPartition(t, int(p)): int(o) for t, parts in state["offsets"].items() for p, o in parts.items()}
        if self._bridges and offs:
            # a replica of a Kafka cluster: the offsets are the cluster's -- commit them there, then
            # mirror afresh from them (the replica may not hold those records any more)
            from ..ops.native import core

            servers, security = self._bridge_spec[0], self._bridge_spec[4]
            client = core().WireClient(servers, "torchkafka-bridge", 30000, security)
            for t in sorted({tp.topic for tp in offs}):
                errs = client.offset_commit(group, t, {tp.partition: o for tp, o in offs.items() if tp.topic == t})
                bad = {p: e for p, e in errs.items() if e}
                if bad:
                    raise KafkaError(f"CommitFailedError: load_state_dict could not commit {t} {bad} on {servers}")
            url = self._bridges[0].url
            for br in reversed(self._bridges):
                br.close(flush=False)
            self._bridges = []
            self._start_bridges(url)
        b = self._broker()
        if offs:
            b.commit(group, offs)
        resumed = {b.pidx(tp.topic, tp.partition): o for tp, o in offs.items()}
        self._committed.update(resumed)
        if int(state.get("version", 1)) == 2:
            # a global-step checkpoint: the steps count on from it, its positions are where every
            # rank stands (each rank's workers start at the committed offsets)
            self._global_step_base = int(state.get("global_step", 0))
            self._steps_delivered = 0
            for pidx, o in resumed.items():
                if o > self._delivered_pos.get(pidx, -1):
                    self._delivered_pos[pidx] = o
