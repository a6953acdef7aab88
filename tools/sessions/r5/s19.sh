# round 5, session 19: what makes an RCCL agreement take ~100 us in the loop (13 us on the device):
# stream priority, words mode, decode streams, torch's NCCL streams
set -o pipefail
O=gpurun_out/r05_s19
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
      "wait/step", r.get("lockstep_wait_us_per_step"), "rtt", t.get("round_trip_us"), "issue", t.get("issue_us"), "wait", t.get("wait_us"), "streams", r["lockstep"].get("streams"))
PY
}
run base ""
run normalprio "TORCHKAFKA_LOCKSTEP_PRIORITY=normal"
run copywords "TORCHKAFKA_RCCL_WORDS=copy"
run hostwords "TORCHKAFKA_RCCL_WORDS=host"
run notorch "TK_BENCH_NO_TORCH_NCCL=1"
run dec1 "TORCHKAFKA_DECODE_STREAMS=1"
run notorch_dec1 "TK_BENCH_NO_TORCH_NCCL=1 TORCHKAFKA_DECODE_STREAMS=1"
run spw32_d32 "" --slots-per-worker 32 --lockstep-depth 32
run spw64_d32 "" --slots-per-worker 64 --lockstep-depth 32
run spw64_d64 "" --slots-per-worker 64 --lockstep-depth 64
echo session done
