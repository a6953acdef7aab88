# RCCL lockstep: 4-word agreements without hipMemcpyAsync, high-priority stream, sync barrier
set -o pipefail
O=gpurun_out/r05_s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_zz_gpu_rccl.py tests/test_gpu_sync_lockstep.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_rccl.log 2>&1 || { tail -40 $O/pytest_rccl.log; exit 1; }
tail -1 $O/pytest_rccl.log
timeout -k 10 120 python tools/probes/queue_probe.py --normal 5 > $O/queue_probe.json 2>&1 || { cat $O/queue_probe.json; exit 1; }
cat $O/queue_probe.json
for m in kernel host copy; do
  TORCHKAFKA_RCCL_WORDS=$m timeout -k 10 400 python bench.py --steps 2000 --extra-blocks rccl,rccl_sync --bridge-steps 0 --config-blocks "" > $O/bench_$m.json 2> $O/bench_$m.err || { tail -20 $O/bench_$m.err; exit 1; }
  python - $O/bench_$m.json $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s, r, y = d["steady_state"], d["steady_rccl"], d["steady_rccl_sync"]
print(sys.argv[2], "steady", s["records_per_s"], "rccl", r["records_per_s"], round(r["records_per_s"] / s["records_per_s"] - 1, 4),
      "commits", r["commits"], "p99", r["commit_latency_p99_us"], "| sync", y["records_per_s"], y["commits"], y["steps"],
      "wait/step", y.get("lockstep_wait_us_per_step"), r["lockstep"].get("words"), r["lockstep"].get("streams", {}).get("shared"))
PY
done
