#!/bin/bash
# One GPU session: build, smoke, GPU tests, bench, rocprof kernel stats.
# Each GPU step has its own time limit; a crash/timeout (124/134/137/139) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $name: stopping"; exit $rc;; esac
  return 0
}
STEPS=${STEPS:-"build smoke bench prof nccl pytest"}
for s in $STEPS; do
  case $s in
    build)  step build 600 python -c "import __graft_entry__ as g; g.build()" ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) step pytest_gpu 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=150 --timeout-method=thread ;;
    nccl)   step nccl_probe 120 python tools/nccl_probe.py ;;
    bench)  step bench 600 python bench.py --stats ;;
    bench8) step bench_fp8 600 python bench.py --stats --dtype fp8 ;;
    prof)   (cd /tmp && export TMPDIR=/tmp && step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$OLDPWD/bench.py" --steps 200) ;;
  esac
done
echo "=== done"
