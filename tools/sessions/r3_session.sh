#!/bin/bash
# Round-3 GPU session: STEPS="smoke benchdrv ..." tools/r3_session.sh
# Each GPU step runs under its own time limit; the first failure (or a crash / time limit) ends the
# script, so nothing more touches the GPU after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${SESSION:-r3}"
mkdir -p "$OUT"
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 12 "$OUT/$name.log" | cut -c1-1500
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
prof() {  # prof <name> <timeout> <rocprofv3 args...> -- <program...>   (kernel trace + stats only)
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$t" rocprofv3 "$@" > "$OUT/$name.log" 2>&1)
  local rc=$?
  tail -n 3 "$OUT/$name.log" | cut -c1-1500
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
pmc() {  # pmc <name> <seconds> <counters...> -- <program...>   (counters only, SIGKILL at the limit)
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL "$t" rocprofv3 --pmc "$@" > "$OUT/$name.log" 2>&1)
  local rc=$?
  tail -n 3 "$OUT/$name.log" | cut -c1-1500
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
R=$PWD
for s in ${STEPS:-smoke benchdrv}; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    pytestk) run pytest_k 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "${PYK}" ;;
    benchdrv) run bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench) run bench 600 python bench.py --stats ;;
    bench2same) run bench_2rank_same 600 python bench.py --gpus 2 --same-device --steps 200 --warmup 50 --steady-steps 4000 --extra-blocks "" ;;
    benchlockr) run bench_lock_rccl 600 python bench.py --lockstep rccl --steps 200 --warmup 50 --steady-steps 8000 --extra-blocks "" ;;
    config4) run config4_w4 300 python benchmarks/config4_json_varlen.py --workers 4 ;;
    config4w8) run config4_w8 300 python benchmarks/config4_json_varlen.py --workers 8 ;;
    config4host) run config4_w4_hostcount 300 python benchmarks/config4_json_varlen.py --workers 4 --json-count host ;;
    config4dma) run config4_w4_dma 300 python benchmarks/config4_json_varlen.py --workers 4 --h2d dma ;;
    config5) run config5 300 python benchmarks/config5_large_messages.py ;;
    bridge) run bridge_e2e 600 python benchmarks/bridge_e2e.py ;;
    profbench) prof profbench 300 --kernel-trace --stats --output-format csv -d "$OUT/profbench" -o run -- python3 "$R/bench.py" --steps 1000 --steady-steps 4000 --extra-blocks "" --bridge-steps 0 ;;
    profdma) prof profdma 300 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/profdma" -o run -- python3 "$R/bench.py" --h2d dma --steps 1000 --steady-steps 4000 --extra-blocks "" --bridge-steps 0 ;;
    pmcspan) pmc pmc_span 120 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_span" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 --steady-steps 0 --extra-blocks "" --bridge-steps 0 ;;
    pmcdma) pmc pmc_dma 120 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_dma" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 --steady-steps 0 --extra-blocks "" --bridge-steps 0 --h2d dma ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
