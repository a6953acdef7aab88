#!/bin/bash
# config 2 steady state, zero-copy decode vs the HBM mirror (h2d='dma'), interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/h2d
for rep in ${REPS:-1 2 3 4}; do
  for h in zerocopy dma; do
    timeout -k 10 200 python bench.py --h2d $h --steps 1000 --extra-blocks "" --bridge-steps 0 > gpurun_out/h2d/${h}_$rep.log 2>&1 || exit $?
    echo "$h rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/h2d/${h}_$rep.log | head -1) $(grep -o '"steady_state": {"steps": [0-9]*, "timed_s": [0-9.]*, "records_per_s": [0-9.]*' gpurun_out/h2d/${h}_$rep.log | grep -o 'records_per_s": [0-9.]*')"
  done
done
