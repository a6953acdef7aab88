# round 5, session 24: the RCCL lockstep at normal priority (its agreements were 2x faster than on a
# high-priority queue in session 19), with more slack
set -o pipefail
O=gpurun_out/r05_s24
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
run() {
  local name=$1 envs=$2; shift 2
  env TORCHKAFKA_LOCKSTEP_TRACE=1 $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks rccl --config-blocks "" --bridge-steps 0 "$@" > $O/$name.json 2> $O/$name.err; local rc=$?
  fatal $rc $name; [ $rc -eq 0 ] || { tail -5 $O/$name.err; return 1; }
  python - $O/$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s, r = d["steady_state"], d["steady_rccl"]
t = r.get("lockstep_trace") or {}
print(sys.argv[2], "steady", round(s["records_per_s"] / 1e6, 1), "rccl", round(r["records_per_s"] / 1e6, 1), round(r["records_per_s"] / s["records_per_s"] - 1, 3),
      "wait/step", r.get("lockstep_wait_us_per_step"), "agreements", r.get("lockstep_agreements"), "rtt", t.get("round_trip_us"), "slack", t.get("slack_us"), "wait", t.get("wait_us"))
PY
}
for i in 1 2; do
  run n_d2_$i "TORCHKAFKA_LOCKSTEP_PRIORITY=normal"
  run n_d8_$i "TORCHKAFKA_LOCKSTEP_PRIORITY=normal" --lockstep-depth 8
  run n_spw64_d32_$i "TORCHKAFKA_LOCKSTEP_PRIORITY=normal" --slots-per-worker 64 --lockstep-depth 32
  run n_host_d8_$i "TORCHKAFKA_LOCKSTEP_PRIORITY=normal TORCHKAFKA_RCCL_WORDS=host" --lockstep-depth 8
done
echo session done
