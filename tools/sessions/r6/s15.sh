# round 6, session 15: where the RCCL block's workers run -- their affinity masks and the CPUs (and
# SMT siblings) they last ran on, in the slow mode (38 us per batch) and the normal one (11-16 us)
set -o pipefail
O=gpurun_out/r06_s15
mkdir -p $O
for rep in 1 2 3 4; do
  n=cpu_$rep
  TK_BENCH_CPU=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 50000 --extra-blocks rccl,shm --config-blocks "" --bridge-steps 0 > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
done
python - <<'PY'
import json, glob
def sib(c):
    try:
        return open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
    except OSError:
        return "?"
for f in sorted(glob.glob("gpurun_out/r06_s15/cpu_*.json")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    for k in ("steady_state", "steady_rccl", "steady_shm"):
        b = j[k]; c = b.get("cpu", {})
        print(f.split("/")[-1], k, round(b["records_per_s"] / 1e6, 2), "fill", b["worker_fill_us_per_batch"], "bpc", b.get("batches_per_commit"),
              "aff", c.get("affinity_of"))
        print("    ", [(t["who"], t["cpu"], sib(t["cpu"]), t["cores"]) for t in c.get("threads", [])[:8]])
PY
echo session done
