#!/bin/bash
# A/B of the HBM-mirror decode kernel time: the tree at _ab/old (byte-table CRC) vs this tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abm
for side in old new; do
  dir=.; [ $side = old ] && dir=_ab/old
  (cd /tmp && export TMPDIR=/tmp && TORCHKAFKA_NO_REBUILD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/abm/$side" -o run -- python3 "$OLDPWD/$dir/bench.py" --h2d dma --steps 1000 --steady-steps 4000 --extra-blocks "" --bridge-steps 0 > "$OLDPWD/gpurun_out/abm/$side.log" 2>&1) || exit $?
  echo "== $side"; grep span_decode gpurun_out/abm/$side/run_kernel_stats.csv | cut -d, -f2-4
  grep -o '"steady_state": {"steps": [0-9]*, "timed_s": [0-9.]*, "records_per_s": [0-9.]*' gpurun_out/abm/$side.log
done
