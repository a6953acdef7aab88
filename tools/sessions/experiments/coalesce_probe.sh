#!/bin/bash
# Group size (batches per decode launch) vs the short (20-step) and steady-state numbers of bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 8 4 2; do
  for rep in 1 2; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --coalesce $c > gpurun_out/coal_${c}_$rep.log 2>&1 || exit 1
    python3 - "$c" gpurun_out/coal_${c}_$rep.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith('{"metric'):
        d = json.loads(line)
        print(f"coalesce {sys.argv[1]}: short {d['value']/1e6:.1f} M  steady {d['steady_state']['records_per_s']/1e6:.1f} M  p99 {d['commit_latency_p99_us']:.0f} us")
PY
  done
done
