#!/bin/bash
# h2d='dma': HBM-mirror copy streams (TORCHKAFKA_MIRROR_COPY_STREAMS) -- tests, then steady rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mcs
timeout -k 10 400 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_loader.py -k "mirror or dma" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/mcs/pytest.log 2>&1 || { tail -30 gpurun_out/mcs/pytest.log; exit 1; }
tail -1 gpurun_out/mcs/pytest.log
for rep in ${REPS:-1 2}; do
  for n in ${NS:-1 2 3}; do
    TORCHKAFKA_MIRROR_COPY_STREAMS=$n timeout -k 10 200 python bench.py --h2d dma --steps 1000 --extra-blocks "" --bridge-steps 0 > gpurun_out/mcs/s${n}_$rep.log 2>&1 || exit $?
    echo "streams $n rep $rep: $(grep -o '"steady_state": {"steps": [0-9]*, "timed_s": [0-9.]*, "records_per_s": [0-9.]*' gpurun_out/mcs/s${n}_$rep.log | grep -o 'records_per_s": [0-9.]*')"
  done
done
