#!/bin/bash
# HBM log mirror (--h2d dma) chunk size x buffers per partition sweep of bench.py's steady state.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 4 8 16; do
  for k in 3 4 6 8; do
    for rep in 1 2; do
      timeout -k 10 120 python bench.py --h2d dma --mirror-chunk-mib $c --mirror-chunks $k --steps 500 \
          > gpurun_out/mirror_${c}_${k}_$rep.log 2>&1 || exit 1
      python3 - "$c" "$k" gpurun_out/mirror_${c}_${k}_$rep.log <<'PY'
import json, sys
for line in open(sys.argv[3]):
    if line.startswith('{"metric'):
        d = json.loads(line)
        print(f"chunk {sys.argv[1]:>2} MiB x {sys.argv[2]}: steady {d['steady_state']['records_per_s']/1e6:.1f} M")
PY
    done
  done
done
