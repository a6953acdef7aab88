#!/bin/bash
# After LogPins::seg_src stopped pinning past the written log end: the GPU suite, then config 4
# through the mirror (REPS runs, default 8) with the in-window pin counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pinfix
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pinfix/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pinfix/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pinfix/pytest_gpu.log
for rep in $(seq 1 "${REPS:-8}"); do
  timeout -k 10 200 python benchmarks/config4_json_varlen.py --h2d dma > gpurun_out/pinfix/c4_$rep.log 2>&1 || exit $?
  echo "config4 dma rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/pinfix/c4_$rep.log) $(grep -o '"log_mib_pinned": [0-9.]*' gpurun_out/pinfix/c4_$rep.log)"
done
