# round 6, session 11: the RCCL block's workers take 38 us per batch against 13 us in the blocks
# around it, at the same CPU (one core each, s10): is it its deeper ring (64 slots per worker against
# 16)?  Every block at 16 and at 64 slots per worker, twice
set -o pipefail
O=gpurun_out/r06_s11
mkdir -p $O
for rep in 1 2; do
  for spw in 16 64; do
    n=spw${spw}_$rep
    TK_BENCH_CPU=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 50000 --extra-blocks rccl,shm --config-blocks "" --bridge-steps 0 --slots-per-worker $spw > $O/$n.json 2> $O/$n.err; rc=$?
    echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_s11/*.json")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    for k in ("steady_state", "steady_rccl", "steady_shm"):
        b = j[k]
        print(f.split("/")[-1], k, round(b["records_per_s"] / 1e6, 2), "slots", b["ring_slots"], "fill", b["worker_fill_us_per_batch"],
              "bpc", b.get("batches_per_commit"), json.dumps(b.get("cpu", {}).get("cores")))
PY
echo session done
