#!/bin/bash
# GPU tests of the decode paths, then the mirror decode's kernel time and rate at the default burst
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mb
timeout -k 10 500 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_loader.py tests/test_gpu_json_span.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/mb/pytest.log 2>&1 || { tail -30 gpurun_out/mb/pytest.log; exit 1; }
tail -1 gpurun_out/mb/pytest.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/mb/prof" -o run -- python3 "$OLDPWD/bench.py" --h2d dma --steps 1000 --steady-steps 4000 --extra-blocks "" --bridge-steps 0 > "$OLDPWD/gpurun_out/mb/prof.log" 2>&1) || exit $?
echo "mirror decode: $(grep span_decode gpurun_out/mb/prof/run_kernel_stats.csv | cut -d, -f2-4)"
timeout -k 10 200 python bench.py --steps 1000 --bridge-steps 0 > gpurun_out/mb/bench.log 2>&1 || exit $?
python - <<'PY'
import json
for l in open('gpurun_out/mb/bench.log'):
    if l.startswith('{"metric'):
        d = json.loads(l)
        print('steady', d['steady_state']['records_per_s'], 'dma', d['steady_dma']['records_per_s'], 'f32', d['steady_f32']['records_per_s'], 'label', d['steady_label']['records_per_s'])
PY
