#!/bin/bash
# After h2d='auto' took the HBM mirror for JSON parsed from the logs: the GPU suite, then config 4
# at its defaults (REPS runs, default 6).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c4auto
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/c4auto/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/c4auto/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/c4auto/pytest_gpu.log
for rep in $(seq 1 "${REPS:-6}"); do
  timeout -k 10 200 python benchmarks/config4_json_varlen.py > gpurun_out/c4auto/c4_$rep.log 2>&1 || exit $?
  echo "config4 auto rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/c4auto/c4_$rep.log) $(grep -o '"decode": "[^"]*"' gpurun_out/c4auto/c4_$rep.log)"
done
