#!/bin/bash
# fixed-width (config 2) ahead depth: the driver-style 20-step value and the 50k-step steady state
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ahead
for a in ${DEPTHS:-2 3 4}; do
  for rep in 1 2; do
    TORCHKAFKA_AHEAD_DEPTH=$a timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --extra-blocks "" --bridge-steps 0 > gpurun_out/ahead/d${a}_$rep.log 2>&1 || exit $?
    python - gpurun_out/ahead/d${a}_$rep.log $a <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric'):
        d = json.loads(l); print('depth', sys.argv[2], 'value', d['value'], 'steady', d['steady_state']['records_per_s'], flush=True)
PY
  done
done
