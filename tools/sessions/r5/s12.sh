# round 5, session 12: new GPU tests (serialized-launch equivalence, teardown without stalls,
# global-step checkpoint, sync lockstep, RCCL), the compressed-bridge and _process blocks, and the
# lockstep depth sweep (the host waited ~1.7 us/step at depth 2)
set -o pipefail
O=gpurun_out/r05_s12
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_teardown.py tests/test_gpu_serialized.py tests/test_gpu_checkpoint.py tests/test_gpu_sync_lockstep.py tests/test_zz_gpu_rccl.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1; rc=$?
tail -15 $O/pytest_new.log; fatal $rc pytest
timeout -k 10 300 python benchmarks/process_override.py > $O/process_override.json 2> $O/process_override.err; rc=$?
tail -c 1500 $O/process_override.json; fatal $rc process
timeout -k 10 600 python bench.py --steps 2000 --extra-blocks "" --config-blocks "" --steady-steps 2000 > $O/bench_bridge.json 2> $O/bench_bridge.err; rc=$?
fatal $rc bridge
python - $O/bench_bridge.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d["bridge"].items():
    if isinstance(v, dict):
        print(k, {x: v[x] for x in v if x in ("records_per_s", "gb_per_s", "compression_ratio", "wire_gb_per_s", "inflated_batches_in_timed_region", "fetch_threads", "inflate_gb_per_s_per_thread", "fetch_thread_time_share", "bridge_errors", "sync_commit_p99_us")})
PY
run() {
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 2000 --extra-blocks rccl --bridge-steps 0 --config-blocks "" "$@" > $O/bench_$name.json 2> $O/bench_$name.err; local rc=$?
  fatal $rc $name
  [ $rc -eq 0 ] || { tail -20 $O/bench_$name.err; return 1; }
  python - $O/bench_$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s, r = d["steady_state"], d["steady_rccl"]
print(sys.argv[2], "steady", s["records_per_s"], "rccl", r["records_per_s"], round(r["records_per_s"] / s["records_per_s"] - 1, 4),
      "agreements", r["lockstep_agreements"], "issue/step", r.get("lockstep_issue_us_per_step"), "wait/step", r.get("lockstep_wait_us_per_step"),
      "p99", r["commit_latency_p99_us"])
PY
}
run d2 "" --lockstep-depth 2
run d8 "" --lockstep-depth 8
run d16 "" --lockstep-depth 16
run d16host "TORCHKAFKA_RCCL_WORDS=host" --lockstep-depth 16
run d32 "" --lockstep-depth 32
echo session done
