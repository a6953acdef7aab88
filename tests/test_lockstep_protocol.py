"""The native cross-rank lockstep (csrc/core/lockstep.h, the credit protocol the GPU step driver
runs) at world 2/4/8 over gloo, with scripted per-rank data paths.

Each rank owns a fake producer with its own record count, arrival pace and ring capacity; the
loop is the driver's: ask the protocol, deliver the oldest staged batch, mark the previous one
finished.  Checked on every rank:
  * all ranks deliver exactly min(batches per rank) steps and stop together (a rank with no
    partitions stops everybody at step 0 instead of hanging them);
  * a rank is never granted a batch it does not hold;
  * a batch becomes committable only after an agreement proves every rank got past it, in
    delivery order, and every delivered batch is committable after finish();
  * a peer that dies makes the others fail within the process-group timeout, not hang.
The reference has no cross-rank notion at all; its per-batch commit orchestration
is auto_commit.py:59-72.
"""
import datetime
import json
import multiprocessing as mp
import os
import random
import socket

import pytest


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Producer:
    """A rank's data path: `total` batches arriving in random bursts, at most `cap` held."""

    def __init__(self, total, cap, seed, slow):
        self.total, self.cap, self.rng, self.slow = total, cap, random.Random(seed), slow
        self.produced = self.delivered = 0

    def _arrive(self, burst):
        room = min(self.cap - (self.produced - self.delivered), self.total - self.produced)
        if room > 0:
            self.produced += min(room, burst)

    def staged(self):
        if not self.slow and self.rng.random() < 0.5:
            self._arrive(self.rng.randrange(1, 4))
        return self.produced - self.delivered

    def all_done(self):
        return self.produced == self.total

    def wait_data(self, timeout_ms):
        if self.slow:
            import time

            time.sleep(0.0005)
        before = self.produced
        self._arrive(self.rng.randrange(1, 3))
        return 1 if self.produced > before else 0


def _rank_main(rank, world, port, outdir, totals, cap, depth, slow_rank, die_rank, sync=False, shared=None,
               fail_at=None):
    import torch
    import torch.distributed as dist

    from torchkafka_amd.ops.native import core

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # a short timeout only where a peer dies on purpose (the survivors must fail, not hang); elsewhere
    # room for slow rank start-up under a loaded test machine (the store waits for rank 0)
    secs = 8 if die_rank >= 0 else 60
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=secs))
    buf = torch.zeros(4, dtype=torch.int64)

    def allreduce_min(a, b, c, d):
        buf[0], buf[1], buf[2], buf[3] = a, b, c, d
        dist.all_reduce(buf, op=dist.ReduceOp.MIN)
        return tuple(int(v) for v in buf.tolist())

    c = core()
    lock = c.CreditLockstep(c.PyLockstepTransport(allreduce_min), depth)
    lock.set_sync(sync)
    committed = []
    lock.set_on_committable(lambda wms: committed.extend(w[1] for w in wms))
    src = _Producer(totals[rank], cap, seed=1000 * rank + depth, slow=(rank == slow_rank))
    out = {"rank": rank, "error": None}
    steps, prev, committed_at_deliver, group_at_deliver = 0, None, [], []
    try:
        while True:
            # the driver's order: asking for the next batch finishes the previous one first
            if prev is not None:
                lock.finished(prev, [(rank, prev, prev + 1, 1)])
                if sync:
                    # the commit of `prev` (what the driver's _sync_commit does), published for the
                    # other ranks to check, and its status for the agreement
                    if shared is not None:
                        shared[rank] = len(committed)
                    if fail_at is not None and fail_at[0] == rank and prev == fail_at[1]:
                        lock.set_commit_status(fail_at[2])
                prev = None
            r = lock.next(src, 20)
            if r == -1:
                continue
            if r == -2:
                break
            assert r == 1, r
            assert src.produced - src.delivered > 0, "granted a batch this rank does not hold"
            idx = lock.delivered()
            assert idx == steps
            src.delivered += 1
            prev = idx
            committed_at_deliver.append(len(committed))
            if shared is not None:
                group_at_deliver.append(min(shared[:]))  # batches every rank committed when idx was handed out
            steps += 1
            if rank == die_rank and steps == 5:
                os._exit(3)  # a crashed peer
        if prev is not None:
            lock.finished(prev, [(rank, prev, prev + 1, 1)])
        lock.finish()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        out["error"] = f"{type(e).__name__}: {e}"
    out.update(steps=steps, committed=committed, committed_at_deliver=committed_at_deliver,
               group_at_deliver=group_at_deliver, agreements=lock.agreements,
               group_commit_failures=lock.group_commit_failures)
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(out, f)
    if out["error"] is None:
        dist.barrier()
        dist.destroy_process_group()


def _run(tmp_path, world, totals, cap=8, depth=2, slow_rank=-1, die_rank=-1, sync=False, fail_at=None):
    # plain processes (not torch's spawn helper, which kills the others when one rank dies)
    port = _free_port()
    ctx = mp.get_context("spawn")
    shared = ctx.Array("q", world, lock=False) if sync else None  # batches each rank committed
    procs = [ctx.Process(target=_rank_main,
                         args=(r, world, port, str(tmp_path), totals, cap, depth, slow_rank, die_rank, sync,
                               shared, fail_at))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=90)
        if p.is_alive():
            p.kill()
            p.join()
    return [json.load(open(tmp_path / f"r{r}.json")) for r in range(world) if (tmp_path / f"r{r}.json").exists()]


@pytest.mark.parametrize("world,totals,cap,depth", [
    (2, [40, 25], 4, 0),
    (2, [60, 60], 2, 2),
    (4, [30, 50, 10, 70], 8, 2),
    (4, [20, 0, 35, 40], 8, 5),        # a rank with no partitions stops everyone at once
    (8, [25, 40, 33, 18, 50, 29, 45, 37], 16, 2),
    (8, [64] * 8, 3, 5),               # tiny ring, deep pipeline
])
def test_credit_lockstep_stops_together_and_commits_only_finished(tmp_path, world, totals, cap, depth):
    res = _run(tmp_path, world, totals, cap=cap, depth=depth, slow_rank=world - 1)
    assert len(res) == world
    want = min(totals)
    for r in res:
        assert r["error"] is None, r["error"]
        assert r["steps"] == want, (r["rank"], r["steps"], want)
        # after finish(): every delivered batch is committable, in delivery order
        assert r["committed"] == list(range(want))
        # while iterating, batch k was never committable before the protocol let k+1 through
        for k, n_committed in enumerate(r["committed_at_deliver"]):
            assert n_committed <= k
        # one agreement grants as many batches as the slowest rank staged: amortised below 1/step
        assert r["agreements"] <= want + 2 + world


@pytest.mark.parametrize("world,totals,cap", [
    (2, [40, 25], 4),
    (2, [30, 30], 2),
    (4, [30, 50, 10, 70], 8),
    (4, [20, 0, 35, 40], 8),           # a rank with no partitions: everyone stops at step 0
    (4, [12, 40, 40, 40], 3),          # one rank runs dry early
])
def test_sync_mode_commits_every_batch_before_the_next_is_delivered(tmp_path, world, totals, cap):
    """commit='sync' under the lockstep (the reference's per-batch commit, auto_commit.py:55-58,
    as an RCCL barrier): each rank commits batch k, then the agreement at step k+1 -- so when batch
    k+1 is handed out on ANY rank, EVERY rank has committed batches 0..k (checked against the
    other ranks' published commit counts, not this rank's)."""
    res = _run(tmp_path, world, totals, cap=cap, depth=2, slow_rank=world - 1, sync=True)
    assert len(res) == world
    want = min(totals)
    for r in res:
        assert r["error"] is None, r["error"]
        assert r["steps"] == want, (r["rank"], r["steps"], want)
        assert r["committed"] == list(range(want))
        # exactly batches 0..k-1 committed here at the moment batch k is delivered ...
        assert r["committed_at_deliver"] == list(range(want)), r["committed_at_deliver"]
        # ... and on every other rank too
        assert r["group_at_deliver"] == list(range(want)), r["group_at_deliver"]
        # one agreement per delivered step (plus starved rounds, the stop and the final barrier)
        assert r["agreements"] >= want
        assert r["group_commit_failures"] == 0


@pytest.mark.parametrize("status,world", [(0, 2), (0, 4), (1, 4)])
def test_sync_mode_a_failed_commit_reaches_every_rank(tmp_path, status, world):
    """A rank whose commit of batch 5 raised (status 0) makes EVERY rank stop with an error at the
    agreement that would hand out batch 6; a swallowed CommitFailedError (status 1, the reference
    logs it and continues, kafka_dataset.py:131-135) lets every rank continue, counted once."""
    res = _run(tmp_path, world, [20] * world, cap=4, depth=2, sync=True, fail_at=(1, 5, status))
    assert len(res) == world
    for r in res:
        if status == 0:
            assert r["error"] is not None and "commit" in r["error"], r
            assert r["steps"] == 6, r  # batches 0..5 handed out, 6 never
        else:
            assert r["error"] is None, r["error"]
            assert r["steps"] == 20
            assert r["group_commit_failures"] == 1


def test_credit_lockstep_peer_death_fails_instead_of_hanging(tmp_path):
    res = _run(tmp_path, 4, [200] * 4, cap=8, depth=2, die_rank=2)
    survivors = [r for r in res if r["rank"] != 2]
    assert len(survivors) == 3
    for r in survivors:
        assert r["error"] is not None, r
