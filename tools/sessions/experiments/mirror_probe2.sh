#!/bin/bash
# After deferring prefetches behind each launch's copy event: mirror depth sweep + the mirror GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_json_span.py -k "mirror" -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_mirror.log 2>&1 || { tail -20 gpurun_out/pytest_mirror.log; exit 1; }
tail -1 gpurun_out/pytest_mirror.log
for k in 4 6 8; do
  for rep in 1 2 3; do
    timeout -k 10 120 python bench.py --h2d dma --mirror-chunks $k --steps 500 > gpurun_out/mirror2_${k}_$rep.log 2>&1 || exit 1
    python3 - "$k" gpurun_out/mirror2_${k}_$rep.log <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith('{"metric'):
        d = json.loads(line)
        print(f"8 MiB x {sys.argv[1]}: head {d['value']/1e6:.1f} steady {d['steady_state']['records_per_s']/1e6:.1f} M")
PY
  done
done
