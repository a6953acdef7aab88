#!/bin/bash
# HBM-mirror stability after the copy marks: mirror GPU tests, VarLen tokens and config 4 through the mirror
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ms2
timeout -k 10 400 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_loader.py -k "mirror or dma" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ms2/pytest.log 2>&1 || { tail -30 gpurun_out/ms2/pytest.log; exit 1; }
tail -1 gpurun_out/ms2/pytest.log
for rep in 1 2 3; do
  timeout -k 10 200 python benchmarks/varlen_tokens.py --h2d dma > gpurun_out/ms2/tok_$rep.log 2>&1 || exit $?
  echo "tokens dma rep $rep: $(grep -o '"value": [0-9]*' gpurun_out/ms2/tok_$rep.log)"
  timeout -k 10 200 python benchmarks/config4_json_varlen.py --h2d dma > gpurun_out/ms2/c4_$rep.log 2>&1 || exit $?
  echo "config4 dma rep $rep: $(grep -o '"value": [0-9]*' gpurun_out/ms2/c4_$rep.log)"
  timeout -k 10 200 python bench.py --h2d dma --steps 1000 --extra-blocks "" --bridge-steps 0 > gpurun_out/ms2/b_$rep.log 2>&1 || exit $?
  echo "bench dma rep $rep: $(grep -o '"steady_state": {"steps": [0-9]*, "timed_s": [0-9.]*, "records_per_s": [0-9.]*' gpurun_out/ms2/b_$rep.log | grep -o 'records_per_s": [0-9.]*')"
done
