"""commit='sync' under the cross-rank lockstep on the native (GPU) step driver: two ranks on one
MI355X over a gloo group (the driver's CreditLockstep in sync mode), agreeing through the group's
all-reduce ('host') or the node-local shared-memory transport ('shm', csrc/core/shm_lockstep.h).
RCCL refuses two ranks on one device, so the RCCL transport is covered at world 1 in
test_zz_gpu_rccl.py.

The reference's contract (auto_commit.py:55-58, kafka_dataset.py:130): batch k's commit completes
before batch k+1 is handed out.  Under DDP that commit is a barrier: each rank commits k, then the
agreement at step k+1 -- so at the moment batch k+1 is yielded on any rank, EVERY rank's part of
batch k is committed (checked across the two ranks' records).
"""
import json
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def batch_ends(x) -> dict:
    """{partition: offset after the batch's last record} from the fixed_f32 rows (col 0 offset, col 1 partition)."""
    v = x.float().cpu()
    out = {}
    for p in v[:, 1].long().unique().tolist():
        out[p] = int(v[v[:, 1] == p][:, 0].max().item()) + 1
    return out


def _rank_main(rank, world, url, port, outdir, verify, transport="host"):
    import torch.distributed as dist

    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit
    from torchkafka_amd.broker.synthetic import open_broker

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class Vec(KafkaDataset):
        schema = FixedWidth(torch.float32, (16,))

    b = open_broker(url)
    dl = DeviceLoader(Vec.placeholder(), 32, num_workers=2, device="cuda:0", dtype=torch.float32, commit="sync",
                      lockstep=transport, verify=verify,
                      worker_init_fn=Vec.init_worker("t", bootstrap_servers=url, group_id="gs",
                                                     auto_offset_reset="earliest", consumer_timeout_ms=500))
    want: dict = {}
    steps, mismatches, snapshots, wants = 0, [], [], []
    for x in auto_commit(dl):
        if steps:
            allc = b.committed_offsets("gs", "t")
            snapshots.append({str(p): o for p, o in allc.items()})
            got = {p: o for p, o in allc.items() if p in want}
            if got != want:
                mismatches.append((steps, got, dict(want)))
        for p, e in batch_ends(x).items():
            want[p] = max(want.get(p, 0), e)
        wants.append({str(p): o for p, o in want.items()})
        steps += 1
    st = dl.stats_summary()
    dl.close()
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump({"steps": steps, "mismatches": mismatches[:3], "snapshots": snapshots, "wants": wants,
                   "commits": st["commits"],
                   "agreements": st["lockstep_agreements"], "lat_p99_us": st["commit_latency_p99_us"]}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("verify,transport", [("deliver", "host"), ("commit", "host"), ("deliver", "shm"),
                                               ("commit", "shm")])
def test_sync_commit_barrier_two_ranks_one_gpu(broker, tmp_path, verify, transport):
    import torch.multiprocessing as tmp

    world = 2
    broker.create_topic("t", 4)
    # rank 0 (partitions 0, 2) has 3 batches of 32 less than rank 1: it runs dry first
    for p in range(4):
        broker.fill("t", 240 - 48 * (p % 2 == 0), "fixed_f32", size=16, partitions=[p], records_per_batch=16)
    ctx = tmp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, broker.url, port, str(tmp_path), verify, transport))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
        if p.is_alive():
            p.kill()
            p.join()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    want_steps = (2 * 192) // 32
    for r in res:
        assert r["steps"] == want_steps, r["steps"]
        assert r["mismatches"] == [], r["mismatches"]
        # every batch committed on its own (one commit per step, the last at the end)
        assert r["commits"] >= want_steps - 1, r["commits"]
    # the cross-rank barrier: when a rank yielded batch k+1, the OTHER rank had committed its batch k
    # too (and possibly k+1, never k+2)
    bad = []
    for r in res:
        for k, snap in enumerate(r["snapshots"]):
            for q in res:
                for p, o in q["wants"][k].items():
                    hi = q["wants"][k + 1][p] if k + 1 < len(q["wants"]) else o
                    if snap.get(p) is None or not o <= snap[p] <= hi:
                        bad.append((k + 1, p, snap.get(p), o, hi))
    assert bad == [], bad[:5]
    committed = broker.committed_offsets("gs", "t")
    assert committed[0] + committed[2] == 384 and committed[1] + committed[3] == 384, committed


def test_shm_lockstep_native_driver_world1_sync_and_async(broker):
    """The node-local shared-memory transport through the native driver at world size 1 (forced
    lockstep='shm' over a world-1 gloo group): sync mode commits every batch before the next is
    handed out; async mode with commit_every=2 commits at least every few batches."""
    import torch.distributed as dist

    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit

    class Vec(KafkaDataset):
        schema = FixedWidth(torch.float32, (8,))

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        broker.create_topic("t", 2)
        broker.fill("t", 400, "fixed_f32", size=8, records_per_batch=10)
        for commit in ("sync", "async"):
            dl = DeviceLoader(Vec.placeholder(), 20, num_workers=2, device="cuda:0", lockstep="shm", commit=commit,
                              dtype=torch.float32, lockstep_commit_every=2,
                              worker_init_fn=Vec.init_worker("t", bootstrap_servers=broker.url, group_id=f"g{commit}",
                                                             auto_offset_reset="earliest", consumer_timeout_ms=300))
            want, steps, lag = {}, 0, []
            for x in auto_commit(dl):
                if steps:
                    got = {p: o for p, o in broker.committed_offsets(f"g{commit}", "t").items() if p in want}
                    lag.append(sum(want[p] - (got.get(p) or 0) for p in want))
                for p, e in batch_ends(x).items():
                    want[p] = max(want.get(p, 0), e)
                steps += 1
            info = dict(dl.lockstep_info)
            st = dl.stats_summary()
            dl.close()
            assert info.get("transport") == "shm", info
            assert steps == 40
            if commit == "sync":
                assert lag == [0] * 39, lag  # batch k committed when k+1 is handed out
            else:
                assert max(lag) <= 20 * 8, lag  # at most a few batches of 20 records behind
                assert st["commits"] >= steps // 4, st["commits"]
            assert broker.committed_offsets(f"g{commit}", "t") == {0: 400, 1: 400}
    finally:
        dist.destroy_process_group()
