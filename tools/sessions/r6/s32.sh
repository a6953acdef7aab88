# round 6, session 32: decode-ahead depth (Tuning.ahead_depth, default 4 groups) against the
# driver's 20-step window, whose closing synchronize drains the groups decoded ahead of it, and
# against the steady state -- depths 1, 2, 4, alternated twice (one box)
set -o pipefail
O=gpurun_out/r06_s32
mkdir -p $O
for rep in 1 2; do
  for d in 1 2 4; do
    n=d${d}_$rep
    TORCHKAFKA_AHEAD_DEPTH=$d timeout -k 10 200 python bench.py --steps 20 --warmup 5 --steady-steps 50000 --extra-blocks "" --config-blocks "" --bridge-steps 0 --window-trace 30 > $O/$n.json 2> $O/$n.err; rc=$?
    echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
    python - "$O/$n.json" "$O/$n.err" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = {}
for line in open(sys.argv[2]):
    if line.startswith('{"window_trace"'):
        w = json.loads(line)["window_trace"]
print("  value", round(j["value"] / 1e6, 2), "steady", round(j["steady_state"]["records_per_s"] / 1e6, 2),
      "window_us", w.get("window_us"), "host_us", w.get("host_us"), "sync_tail_us", w.get("sync_tail_us"))
PY
  done
done
echo session done
