#!/bin/bash
# h2d='dma' decode: LDS-DMA loads in flight per wave (TORCHKAFKA_SPAN_BURST) -- kernel time and rate
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/burst
for b in ${BURSTS:-1 0 4}; do
  (cd /tmp && export TMPDIR=/tmp && TORCHKAFKA_SPAN_BURST=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/burst/b$b" -o run -- python3 "$OLDPWD/bench.py" --h2d dma --steps 1000 --steady-steps 4000 --extra-blocks "" --bridge-steps 0 > "$OLDPWD/gpurun_out/burst/b$b.log" 2>&1) || exit $?
  echo "burst $b: $(grep span_decode gpurun_out/burst/b$b/run_kernel_stats.csv | cut -d, -f2-4)"
  TORCHKAFKA_SPAN_BURST=$b timeout -k 10 200 python bench.py --h2d dma --steps 1000 --extra-blocks "" --bridge-steps 0 > gpurun_out/burst/rate$b.log 2>&1 || exit $?
  echo "burst $b rate: $(grep -o '"steady_state": {"steps": [0-9]*, "timed_s": [0-9.]*, "records_per_s": [0-9.]*' gpurun_out/burst/rate$b.log)"
done
