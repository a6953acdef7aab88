#!/bin/bash
# config 4 kernel traces: device counting vs worker counting (json_count=host)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for jc in device host; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/profc4_$jc" -o run -- python3 "$OLDPWD/benchmarks/config4_json_varlen.py" --steps 4000 --json-count $jc > "$OLDPWD/gpurun_out/profc4_$jc.log" 2>&1) || exit $?
  echo "== $jc"; grep -o '"value": [0-9]*' gpurun_out/profc4_$jc.log
  cut -d, -f1-4 gpurun_out/profc4_$jc/run_kernel_stats.csv | cut -c1-150 | head -4
done
for jc in device host; do
  timeout -k 10 200 python benchmarks/config4_json_varlen.py --steps 20000 --json-count $jc > gpurun_out/c4_$jc.log 2>&1 || exit $?
  echo "== plain $jc"; grep -o '"value": [0-9]*\|"worker_fill_us_per_batch": [0-9.]*\|"json_width_wait_us_per_batch": [0-9.]*' gpurun_out/c4_$jc.log
done
