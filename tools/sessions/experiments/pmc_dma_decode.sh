#!/bin/bash
# PMC pass over the HBM-mirror decode (h2d='dma'): where a span_decode workgroup's cycles go
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE --output-format csv -d "$OLDPWD/gpurun_out/pmc_dma" -o run -- python3 "$OLDPWD/bench.py" --h2d dma --steps 300 --warmup 20 --steady-steps 0 --extra-blocks "" --bridge-steps 0 > "$OLDPWD/gpurun_out/pmc_dma.log" 2>&1) || exit $?
python - <<'PY'
import csv, collections
agg = collections.defaultdict(float)
n = collections.Counter()
for r in csv.DictReader(open('gpurun_out/pmc_dma/run_counter_collection.csv')):
    if 'span_decode' in r['Kernel_Name']:
        agg[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
print({k: round(v) for k, v in agg.items()}, n['SQ_WAVES'])
PY
