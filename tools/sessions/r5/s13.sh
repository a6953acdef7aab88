# round 5, session 13: the bridge blocks (which stalled in s12) with a stack watchdog; the teardown
# test; the 20-step headline window (driver command shape) with its trace; the lockstep depth sweep
set -o pipefail
O=gpurun_out/r05_s13
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
TK_BENCH_WATCHDOG=45 timeout -k 10 280 python bench.py --steps 2000 --extra-blocks "" --config-blocks "" --steady-steps 2000 > $O/bench_bridge.json 2> $O/bench_bridge.err; rc=$?
grep -v "amdgpu.ids" $O/bench_bridge.err | head -c 6000; fatal $rc bridge
python - $O/bench_bridge.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d["bridge"].items():
    if isinstance(v, dict):
        print(k, {x: v[x] for x in v if x in ("records_per_s", "gb_per_s", "compression_ratio", "wire_gb_per_s", "inflated_batches_in_timed_region", "fetch_threads", "inflate_gb_per_s_per_thread", "fetch_thread_time_share", "bridge_errors", "sync_commit_p99_us")})
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_teardown.py -v -s -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_teardown.log 2>&1; rc=$?
tail -5 $O/pytest_teardown.log; fatal $rc teardown
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-blocks "" --config-blocks "" --bridge-steps 0 --steady-steps 0 --window-trace 20 > $O/head_$i.json 2> $O/head_$i.err; rc=$?; fatal $rc head
  python -c "import json,sys; d=json.loads(open('$O/head_$i.json').read().strip().splitlines()[-1]); print('head', d['value'], d['ms_per_step'])"
  grep -o '"window_us": [0-9.]*\|"host_us": [0-9.]*\|"sync_tail_us": [0-9.]*' $O/head_$i.err | tr '\n' ' '; echo
done
for c in 4 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-blocks "" --config-blocks "" --bridge-steps 0 --steady-steps 20000 --window-trace 20 --coalesce $c > $O/head_c$c.json 2> $O/head_c$c.err; rc=$?; fatal $rc headc
  python -c "import json,sys; d=json.loads(open('$O/head_c$c.json').read().strip().splitlines()[-1]); print('coalesce $c head', d['value'], 'steady', d['steady_state']['records_per_s'])"
  grep -o '"window_us": [0-9.]*\|"host_us": [0-9.]*\|"sync_tail_us": [0-9.]*' $O/head_c$c.err | tr '\n' ' '; echo
done
run() {
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py --steps 2000 --extra-blocks rccl --bridge-steps 0 --config-blocks "" "$@" > $O/bench_$name.json 2> $O/bench_$name.err; local rc=$?
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
echo session done
