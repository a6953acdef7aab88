# round 5, session 18: where an RCCL agreement's round trip goes (host timestamps), at depth 2 and 16
set -o pipefail
O=gpurun_out/r05_s18
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for d in 2 16; do
  TORCHKAFKA_LOCKSTEP_TRACE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks rccl --config-blocks "" --bridge-steps 0 --lockstep-depth $d > $O/bench_d$d.json 2> $O/bench_d$d.err; rc=$?
  fatal $rc d$d; [ $rc -eq 0 ] || { tail -5 $O/bench_d$d.err; exit 1; }
  python - $O/bench_d$d.json $d <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s, r = d["steady_state"], d["steady_rccl"]
print("depth", sys.argv[2], "steady", s["records_per_s"], "rccl", r["records_per_s"], round(r["records_per_s"] / s["records_per_s"] - 1, 4),
      "wait/step", r.get("lockstep_wait_us_per_step"), r.get("lockstep_trace"))
PY
done
echo session done
