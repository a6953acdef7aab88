#!/bin/bash
# JSON device path: GPU tests, then config 4 (4 workers)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_json_span.py tests/test_gpu_json_parse.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_json.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_json.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python benchmarks/config4_json_varlen.py > gpurun_out/config4.log 2>&1 || exit $?
python - <<'PY'
import json
for l in open('gpurun_out/config4.log'):
    if l.startswith('{'):
        d = json.loads(l); L = d['loader']
        print(d['value'], d['workers'], {k: round(L[k], 2) for k in ('host_issue_us_per_batch', 'worker_fill_us_per_batch', 'native_launch_us_per_step', 'ahead_launch_us_per_batch', 'json_width_wait_us_per_batch')})
PY
