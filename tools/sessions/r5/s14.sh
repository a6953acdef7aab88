# round 5, session 14: the driver's command with every default block (timed), then the RCCL
# lockstep cost at the default depth three more times
set -o pipefail
O=gpurun_out/r05_s14
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
t0=$(date +%s)
TK_BENCH_WATCHDOG=120 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err; rc=$?
echo "driver-style bench rc=$rc wall=$(( $(date +%s) - t0 )) s"; grep "^\[bench\]" $O/bench_driver.err; fatal $rc driver
python - $O/bench_driver.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "steady", d["steady_state"]["records_per_s"])
for k in ("steady_dma", "steady_f32", "steady_label", "steady_rccl", "steady_rccl_sync", "steady_unverified"):
    if k in d: print(k, d[k]["records_per_s"], d[k].get("commit"), d[k].get("batches_per_commit"))
for k, v in (d.get("bridge") or {}).items():
    if isinstance(v, dict): print("bridge", k, v["records_per_s"], v.get("gb_per_s"))
for k in ("steady_compute", "config4", "config5", "config1", "process_override"):
    if k in d: print(k, json.dumps(d[k])[:600])
PY
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 2000 --extra-blocks rccl,rccl_sync --bridge-steps 0 --config-blocks "" > $O/bench_rccl_$i.json 2> $O/bench_rccl_$i.err; rc=$?
  fatal $rc rccl
  python - $O/bench_rccl_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s, r, q = d["steady_state"], d["steady_rccl"], d["steady_rccl_sync"]
print("steady", s["records_per_s"], "rccl", r["records_per_s"], round(r["records_per_s"] / s["records_per_s"] - 1, 4),
      "wait/step", r.get("lockstep_wait_us_per_step"), "| sync", q["records_per_s"], q["commits"], q["steps"])
PY
done
echo session done
