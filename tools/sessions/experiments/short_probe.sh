#!/bin/bash
# Short-run headline probe: bench.py --steps 20 --warmup 5 under worker-spin / ahead-depth variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "a:" "b:TORCHKAFKA_WORKER_SPIN_US=100000" "c:TORCHKAFKA_AHEAD_DEPTH=8"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --stats --steady-steps 0 \
      > gpurun_out/short_$n.log 2>&1 || exit 1
  echo "== $n $e"
  grep -o '"value": [0-9.]*\|"timed_region_s": [0-9.]*' gpurun_out/short_$n.log | tr '\n' ' '; echo
  grep -o '"native_[a-z]*_us_per_step": [0-9.]*\|"host_wait_us_per_batch": [0-9.]*\|"slots_on_gpu_avg": [0-9.]*\|"group_launches_per_batch": [0-9.]*' gpurun_out/short_$n.log | tr '\n' ' '; echo
done
