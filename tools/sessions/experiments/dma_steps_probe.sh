#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for st in 500 2000; do
  for k in 4 6; do
    for rep in 1 2; do
      timeout -k 10 120 python bench.py --h2d dma --mirror-chunks $k --steps $st --stats > gpurun_out/dmast_${st}_${k}_$rep.log 2>&1 || exit 1
      python3 - "$st" "$k" gpurun_out/dmast_${st}_${k}_$rep.log <<'PY'
import json, sys
st = {}
for line in open(sys.argv[3]):
    if line.startswith('{"loader_stats'):
        st = json.loads(line)["loader_stats"]
    if line.startswith('{"metric'):
        d = json.loads(line)
        print(f"steps {sys.argv[1]} K {sys.argv[2]}: head {d['value']/1e6:.1f} steady {d['steady_state']['records_per_s']/1e6:.1f} M "
              f"fallbacks {st.get('mirror_fallbacks')} copies {st.get('mirror_copies')} pin_ms {st.get('log_pin_ms', 0):.0f}")
PY
    done
  done
done
