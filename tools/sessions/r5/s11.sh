# lockstep cost: decode-stream priority / count under the RCCL lockstep; high-priority queue pool
set -o pipefail
O=gpurun_out/r05_s11
mkdir -p $O
for hp in 1 2 3 4; do timeout -k 10 60 python tools/probes/queue_probe.py --normal 3 --high-pool $hp 2>/dev/null | tail -1; done > $O/queue_probe.json || exit 1
cat $O/queue_probe.json
run() {
  local name=$1 envs=$2
  env $envs timeout -k 10 400 python bench.py --steps 2000 --extra-blocks rccl,rccl_sync --bridge-steps 0 --config-blocks "" > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; return 1; }
  python - $O/bench_$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s, r, y = d["steady_state"], d["steady_rccl"], d["steady_rccl_sync"]
print(sys.argv[2], "steady", s["records_per_s"], "rccl", r["records_per_s"], round(r["records_per_s"] / s["records_per_s"] - 1, 4),
      "agreements", r["lockstep_agreements"], "issue/step", r.get("lockstep_issue_us_per_step"), "wait/step", r.get("lockstep_wait_us_per_step"),
      "| sync", y["records_per_s"], y["commits"], "issue/step", y.get("lockstep_issue_us_per_step"), "wait/step", y.get("lockstep_wait_us_per_step"),
      r["lockstep"].get("streams"))
PY
}
run base "" || exit 1
run hi3 "TORCHKAFKA_DECODE_PRIORITY=high TORCHKAFKA_DECODE_STREAMS=3" || exit 1
run hi3host "TORCHKAFKA_DECODE_PRIORITY=high TORCHKAFKA_DECODE_STREAMS=3 TORCHKAFKA_RCCL_WORDS=host" || exit 1
run n3 "TORCHKAFKA_DECODE_STREAMS=3" || exit 1
