#!/bin/bash
# JSON / var-len device decode with the mirror default: GPU tests, config 4, tokens zero-copy vs dma
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/jm
timeout -k 10 500 python -u -m pytest tests/test_gpu_json_span.py tests/test_gpu_json_parse.py tests/test_gpu_span.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/jm/pytest.log 2>&1 || { tail -30 gpurun_out/jm/pytest.log; exit 1; }
tail -1 gpurun_out/jm/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python benchmarks/config4_json_varlen.py --steps 20000 > gpurun_out/jm/c4_$rep.log 2>&1 || exit $?
  echo "config4 auto rep $rep: $(grep -o '"value": [0-9]*, "ms_per_step\|"decode": "[^"]*"' gpurun_out/jm/c4_$rep.log | tr '\n' ' ')"
  for h in auto dma; do
    timeout -k 10 200 python benchmarks/varlen_tokens.py --h2d $h > gpurun_out/jm/tok_${h}_$rep.log 2>&1 || exit $?
    echo "tokens $h rep $rep: $(grep -o '"value": [0-9]*' gpurun_out/jm/tok_${h}_$rep.log)"
  done
done
