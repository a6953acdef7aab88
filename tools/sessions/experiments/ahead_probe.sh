#!/bin/bash
# Decode-ahead depth vs the short (20-step) and steady-state numbers of bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for a in 4 6 8 12; do
  for spw in 16 32; do
    TORCHKAFKA_AHEAD_DEPTH=$a timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --slots-per-worker $spw \
        > gpurun_out/ahead_${a}_$spw.log 2>&1 || exit 1
    python3 - "$a" "$spw" gpurun_out/ahead_${a}_$spw.log <<'PY'
import json, sys
for line in open(sys.argv[3]):
    if line.startswith('{"metric'):
        d = json.loads(line)
        print(f"ahead {sys.argv[1]:>2} spw {sys.argv[2]}: short {d['value']/1e6:.1f} M  steady {d['steady_state']['records_per_s']/1e6:.1f} M  p99 {d['commit_latency_p99_us']:.0f} us")
PY
  done
done
