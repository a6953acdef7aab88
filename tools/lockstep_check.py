"""Multi-rank check of the native driver's lockstep protocol on ONE GPU.

Launch: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
            tools/lockstep_check.py [--transport host|rccl]
Every rank uses cuda:0 for the device path; the per-step agreement goes through
gloo (``lockstep="host"``) by default.  ``LOCKCHECK_TRANSPORT=rccl`` tries the native
RCCL transport instead (two ranks on one GPU: only if RCCL accepts that).  Rank r owns
partitions {r, r + world}; the last rank has the least data, so every rank must
stop at its batch count, and only batches all ranks finished may be committed.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import faulthandler

    faulthandler.dump_traceback_later(75, exit=True)  # a hang prints every thread's stack
    import torch
    import torch.distributed as dist

    from torchkafka_amd import DeviceLoader, FixedWidth, JsonArray, KafkaDataset, auto_commit
    from torchkafka_amd.broker import SyntheticBroker

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    url = f"shm://tklockcheck-{os.getppid()}"
    b = SyntheticBroker.create(url)
    n_parts = 2 * world
    b.create_topic("t", n_parts)
    per_rank = [100 - 20 * (r == world - 1) for r in range(world)]
    json_mode = os.environ.get("LOCKCHECK_SCHEMA", "fixed") == "json"  # device JSON parse path
    if json_mode:
        b.fill("t", per_rank[rank] // 2, "json_f32", size=2, max_size=12, partitions=[rank, rank + world])
    else:
        b.fill("t", per_rank[rank] // 2, "fixed_f32", size=8, partitions=[rank, rank + world])
    dist.init_process_group("gloo")
    dist.barrier()

    class Vec(KafkaDataset):
        schema = JsonArray() if json_mode else FixedWidth(torch.float32, (8,))

    results = {}
    depths = [int(d) for d in os.environ.get("LOCKCHECK_DEPTHS", "0,2,5").split(",")]
    for depth in depths:
        group = f"g{depth}"
        dl = DeviceLoader(Vec.placeholder(), 10, num_workers=2, device="cuda:0",
                          lockstep=os.environ.get("LOCKCHECK_TRANSPORT", "host"),
                          lockstep_depth=depth,
                          worker_init_fn=Vec.init_worker("t", bootstrap_servers=url, group_id=group,
                                                         auto_offset_reset="earliest", consumer_timeout_ms=500))
        steps, parts = 0, set()
        print(f"[rank {rank}] depth {depth}: iterating", flush=True)
        for x in auto_commit(dl):
            steps += 1
            print(f"[rank {rank}] depth {depth}: step {steps}", flush=True)
            if json_mode:
                parts = {rank, rank + world}  # rows carry no partition id; the commits below check it
            else:
                parts |= set(x[:, 1].long().tolist())
        torch.cuda.synchronize()
        dist.barrier()
        committed = b.committed_offsets(group, "t")
        mine = committed[rank] + committed[rank + world]
        results[depth] = (steps, sorted(parts), mine)
        assert steps == 8, (rank, depth, steps)
        assert sorted(parts) == [rank, rank + world], (rank, parts)
        assert mine == 80, (rank, depth, committed)
    print(json.dumps({"rank": rank, "ok": True, "results": results}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        b.destroy()


if __name__ == "__main__":
    main()
