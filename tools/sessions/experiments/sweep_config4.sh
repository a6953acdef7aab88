#!/bin/bash
# config 4 knob sweep, 20000 timed steps each (one box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c4sweep
one() {  # one <name> <env...> -- args
  local name=$1; shift
  env "$@" timeout -k 10 200 python benchmarks/config4_json_varlen.py --steps 20000 > gpurun_out/c4sweep/$name.log 2>&1 || exit $?
  python - gpurun_out/c4sweep/$name.log "$name" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); L = d['loader']
        print(sys.argv[2], d['value'], {k: round(L.get(k, -1), 2) for k in ('host_issue_us_per_batch', 'worker_fill_us_per_batch', 'ahead_launch_us_per_batch', 'json_width_wait_us_per_batch', 'native_next_us_per_step')}, flush=True)
PY
}
timeout -k 10 400 python -u -m pytest tests/test_gpu_json_span.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_json.log 2>&1 || { tail -30 gpurun_out/pytest_json.log; exit 1; }
tail -2 gpurun_out/pytest_json.log
for s in ${SWEEP:-base base2}; do
  case $s in
    base*) one $s TK_X=1 ;;
    ahead*) one $s TORCHKAFKA_AHEAD_DEPTH=${s#ahead} ;;
    streams*) one $s TORCHKAFKA_DECODE_STREAMS=${s#streams} ;;
  esac
done
