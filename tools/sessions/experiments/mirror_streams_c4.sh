#!/bin/bash
# Config 4 through the HBM mirror (h2d=dma) at 1, 2 and 4 copy streams, 3 runs each: how often a
# run collapses, and whether more copy streams (shorter per-stream prefetch queues) change that.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/msc4
for rep in 1 2 3; do
  for s in 1 2 4; do
    TORCHKAFKA_MIRROR_COPY_STREAMS=$s timeout -k 10 200 python benchmarks/config4_json_varlen.py --h2d dma > gpurun_out/msc4/c4_s${s}_$rep.log 2>&1 || exit $?
    echo "config4 dma streams=$s rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/msc4/c4_s${s}_$rep.log)"
  done
done
