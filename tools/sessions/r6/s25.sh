# round 6, session 25: the driver's N = 4 command rehearsed again as four ranks on this GPU, every
# default block but RCCL's (session 18's failed in the dma block), then session 19's census of the
# compressed bridge blocks.
set -o pipefail
O=gpurun_out/r06_s25
mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29653 bench.py --gpus 4 --same-device --steps 20 --warmup 5 > $O/four_rank.json 2> $O/four_rank.err; rc=$?
grep "^\[bench\]" $O/four_rank.err | tail -30 > $O/four_rank_progress.txt; cat $O/four_rank_progress.txt; echo "four-rank rc=$rc"; [ $rc -eq 0 ] || { tail -8 $O/four_rank.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_s25/four_rank.json").read().strip().splitlines()[-1])
out = {k: d[k] for k in ("value", "n_gpus", "ms_per_step") if k in d}
for k, v in list(d.items()) + [("bridge_" + k, v) for k, v in (d.get("bridge") or {}).items()]:
    if isinstance(v, dict) and ("records_per_s" in v or "error" in v):
        out[k] = v.get("error") or (round(v["records_per_s"] / 1e6, 2), v.get("batches_per_commit"))
print(json.dumps(out)[:3000])
PY
bash tools/sessions/r6/s19.sh
