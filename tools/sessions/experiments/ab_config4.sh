#!/bin/bash
# A/B of config 4 between the tree at _bisect/old and this tree (same box), then a kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
summ() {
python - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); L = d['loader']
        print(sys.argv[1], d['value'], {k: round(L.get(k, -1), 2) for k in ('host_issue_us_per_batch', 'native_launch_us_per_step', 'ahead_launch_us_per_batch', 'json_width_wait_us_per_batch')})
PY
}
for rep in 1 2; do
  (cd _bisect/old && TORCHKAFKA_NO_REBUILD=1 timeout -k 10 200 python benchmarks/config4_json_varlen.py > ../../gpurun_out/ab_old_$rep.log 2>&1) || exit $?
  summ gpurun_out/ab_old_$rep.log
  TORCHKAFKA_NO_REBUILD=1 timeout -k 10 200 python benchmarks/config4_json_varlen.py > gpurun_out/ab_new_$rep.log 2>&1 || exit $?
  summ gpurun_out/ab_new_$rep.log
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/profc4" -o run -- python3 "$OLDPWD/benchmarks/config4_json_varlen.py" --steps 2000 > "$OLDPWD/gpurun_out/profc4.log" 2>&1) || exit $?
cut -d, -f1-4 gpurun_out/profc4/run_kernel_stats.csv | cut -c1-150
