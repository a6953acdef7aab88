#!/bin/bash
# Config 4, zero-copy against the HBM mirror (h2d=dma, 2 copy streams), alternated on one box,
# REPS runs each (default 10): the distribution of each, collapses included.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abc4
for rep in $(seq 1 "${REPS:-10}"); do
  for h in zerocopy dma; do
    timeout -k 10 200 python benchmarks/config4_json_varlen.py --h2d $h > gpurun_out/abc4/c4_${h}_$rep.log 2>&1 || exit $?
    echo "config4 $h rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/abc4/c4_${h}_$rep.log)"
  done
done
