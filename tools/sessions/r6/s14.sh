# round 6, session 14: the RCCL async block with one decode stream (fitted to the 4 hardware
# queues, the default) against two (round 5's layout: a decode stream shares a queue), alternated
set -o pipefail
O=gpurun_out/r06_s14
mkdir -p $O
for rep in 1 2 3; do
  for ds in fit 2; do
    extra=""; [ $ds = 2 ] && extra="--decode-streams 2"
    n=rccl_ds${ds}_$rep
    TK_BENCH_CPU=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 50000 --extra-blocks rccl $extra --config-blocks "" --bridge-steps 0 > $O/$n.json 2> $O/$n.err; rc=$?
    echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_s14/*.json")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    for k in ("steady_state", "steady_rccl"):
        b = j[k]
        print(f.split("/")[-1], k, round(b["records_per_s"] / 1e6, 2), "fill", b["worker_fill_us_per_batch"], "bpc", b.get("batches_per_commit"),
              "agr", b.get("lockstep_agreements"), (b.get("lockstep") or {}).get("streams", {}).get("decode"))
PY
echo session done
