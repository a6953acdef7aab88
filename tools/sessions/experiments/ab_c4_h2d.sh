#!/bin/bash
# config 4 (4 workers, 20 000 steps): zero-copy vs the HBM mirror, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c4h
for rep in 1 2; do
  for h in auto dma; do
    timeout -k 10 200 python benchmarks/config4_json_varlen.py --steps 20000 --h2d $h > gpurun_out/c4h/${h}_$rep.log 2>&1 || exit $?
    python - gpurun_out/c4h/${h}_$rep.log $h <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); L = d['loader']
        print(sys.argv[2], d['value'], d['decode'], {k: round(L.get(k, -1), 2) for k in ('host_issue_us_per_batch', 'worker_fill_us_per_batch', 'json_width_wait_us_per_batch', 'mirror_mib_copied')}, flush=True)
PY
  done
done
