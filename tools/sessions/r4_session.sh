#!/bin/bash
# Round-4 GPU session: STEPS="smoke benchdrv ..." SESSION=name tools/r4_session.sh
# (steps of one-off A/Bs that were reverted were removed; their logs are under profiles/r04_*)
# Each GPU step runs under its own time limit; the first failure (or a crash / time limit) ends the
# script, so nothing more touches the GPU after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${SESSION:-r4}"
mkdir -p "$OUT"
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 12 "$OUT/$name.log" | cut -c1-1500
  echo "=== $name rc=$rc"
  # a failed test or bench is recorded and the session goes on; a crash, abort or time limit
  # (124/134/137/139) ends it: nothing more touches the GPU after a fault
  case $rc in 0) ;; 124|134|137|139) exit $rc ;; *) FAILED="$FAILED $name" ;; esac
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
FAILED=""
trap 'echo "=== failed steps:${FAILED:- none}"' EXIT
for s in ${STEPS:-smoke benchdrv}; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    pytestk) run pytest_k 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "${PYK}" ;;
    benchdrv) run bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench) run bench 600 python bench.py --stats ;;
    bench2same) run bench_2rank_same 600 python bench.py --gpus 2 --same-device --steps 200 --warmup 50 --steady-steps 4000 --extra-blocks "" ;;
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
    benchlockr) run bench_lock_rccl 600 python bench.py --lockstep rccl --steps 200 --warmup 50 --steady-steps 50000 --extra-blocks "" --bridge-steps 0 ;;
    benchplain) run bench_plain 600 python bench.py --steps 200 --warmup 50 --steady-steps 50000 --extra-blocks "" --bridge-steps 0 ;;
    profrccl) prof profrccl 300 --kernel-trace --hip-trace --stats --output-format csv -d "$OUT/profrccl" -o run -- python3 "$R/bench.py" --lockstep rccl --steps 1000 --steady-steps 8000 --extra-blocks "" --bridge-steps 0 ;;
    profplain) prof profplain 300 --kernel-trace --hip-trace --stats --output-format csv -d "$OUT/profplain" -o run -- python3 "$R/bench.py" --steps 1000 --steady-steps 8000 --extra-blocks "" --bridge-steps 0 ;;
    pytestnew) run pytest_new 600 python -u -m pytest tests/test_gpu_sync_lockstep.py tests/test_gpu_span.py tests/test_gpu_loader.py tests/test_multirank_launch.py -k "sync or verify or parse_error or launcher" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    pytestrccl) run pytest_rccl 300 python -u -m pytest tests/test_zz_gpu_rccl.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    benchverify) run bench_verify_commit 600 python bench.py --verify commit --steps 200 --warmup 50 --steady-steps 50000 --extra-blocks "" --bridge-steps 0 ;;
    pytestpin) run pytest_pin 600 python -u -m pytest tests/test_gpu_span.py -k "pins_only or growing_log or mirror" -x -v -p no:cacheprovider --timeout 180 --timeout-method thread ;;
    c4mirror) for rep in $(seq 1 "${REPS:-12}"); do run c4_dma_$rep 200 python benchmarks/config4_json_varlen.py --h2d dma; grep -o '"value": [0-9]*' "$OUT/c4_dma_$rep.log"; grep -o '"log_pin_ms": [0-9.]*\|"log_pin_wait_ms": [0-9.]*\|"log_mib_pinned": [0-9.]*' "$OUT/c4_dma_$rep.log" | tr '\n' ' '; echo; done ;;
    c4zc) for rep in $(seq 1 "${REPS:-12}"); do run c4_zc_$rep 200 python benchmarks/config4_json_varlen.py; grep -o '"value": [0-9]*' "$OUT/c4_zc_$rep.log"; done ;;
    tokens) run tokens_zc 300 python benchmarks/varlen_tokens.py && run tokens_dma 300 python benchmarks/varlen_tokens.py --h2d dma ;;
    c4wait) for rep in $(seq 1 "${REPS:-4}"); do TORCHKAFKA_MIRROR_WAIT=1 run c4_wait_$rep 200 python benchmarks/config4_json_varlen.py --h2d dma; grep -o '"value": [0-9]*' "$OUT/c4_wait_$rep.log"; done ;;
    c5ab) for rep in 1 2; do run c5_deliver_$rep 200 python benchmarks/config5_large_messages.py && run c5_commit_$rep 200 python benchmarks/config5_large_messages.py --verify commit; done ;;
    prof4) prof prof4 300 --kernel-trace --hip-trace --stats --output-format csv -d "$OUT/prof4" -o run -- python3 "$R/benchmarks/config4_json_varlen.py" --h2d dma ;;
    prof4zc) prof prof4zc 300 --kernel-trace --hip-trace --stats --output-format csv -d "$OUT/prof4zc" -o run -- python3 "$R/benchmarks/config4_json_varlen.py" ;;
    c5) for rep in 1 2 3; do run c5_deliver_$rep 200 python benchmarks/config5_large_messages.py; grep -o '"value": [0-9.]*' "$OUT/c5_deliver_$rep.log"; done ;;
    pytestjson) run pytest_json 600 python -u -m pytest tests/test_gpu_json_span.py tests/test_gpu_json_parse.py tests/test_gpu_span.py tests/test_gpu_loader.py -k "json or verify or count or span" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    benchahead) for d in 0 1 2 4 0 1 2 4; do TORCHKAFKA_AHEAD_DEPTH=$d run bench_ahead${d}_$RANDOM 300 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks "" --bridge-steps 0 --config-blocks ""; done; grep -o '"value": [0-9.]*\|"records_per_s": [0-9.]*' "$OUT"/bench_ahead*.log ;;
    pmcjson) pmc pmc_json 120 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_json" -o run -- python3 "$R/benchmarks/config4_json_varlen.py" --steps 3000 ;;
    profjson) prof profjson 300 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/profjson" -o run -- python3 "$R/benchmarks/config4_json_varlen.py" ;;
    launchcost) run launch_cost 60 tools/probes/launch_cost_probe ;;
    pytestq) TORCHKAFKA_HIP_QUEUE=1 run pytest_queue 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread ;;
    abqueue) for rep in 1 2 3; do
            run c4_base_$rep 200 python benchmarks/config4_json_varlen.py &&
            TORCHKAFKA_HIP_QUEUE=1 run c4_q_$rep 200 python benchmarks/config4_json_varlen.py
          done
          for rep in 1 2; do
            run bench_base_$rep 300 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks "" --bridge-steps 0 --config-blocks "" &&
            TORCHKAFKA_HIP_QUEUE=1 run bench_q_$rep 300 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks "" --bridge-steps 0 --config-blocks ""
          done
          run tokens_base 300 python benchmarks/varlen_tokens.py && TORCHKAFKA_HIP_QUEUE=1 run tokens_q 300 python benchmarks/varlen_tokens.py
          run c5_base 200 python benchmarks/config5_large_messages.py && TORCHKAFKA_HIP_QUEUE=1 run c5_q 200 python benchmarks/config5_large_messages.py
          grep -o '"value": [0-9.]*' "$OUT"/c4_*.log "$OUT"/bench_*.log "$OUT"/tokens_*.log "$OUT"/c5_*.log ;;
    abvalue) for rep in 1 2 3 4; do
            run bv_q_$rep 300 python bench.py --steps 20 --warmup 5 --steady-steps 8000 --extra-blocks "" --bridge-steps 0 --config-blocks "" &&
            TORCHKAFKA_HIP_QUEUE=0 run bv_base_$rep 300 python bench.py --steps 20 --warmup 5 --steady-steps 8000 --extra-blocks "" --bridge-steps 0 --config-blocks ""
          done
          for rep in 1 2 3; do
            run c4_q_$rep 200 python benchmarks/config4_json_varlen.py && TORCHKAFKA_HIP_QUEUE=0 run c4_base_$rep 200 python benchmarks/config4_json_varlen.py
          done
          grep -o '"value": [0-9.]*\|"timed_region_s": [0-9.]*' "$OUT"/bv_*.log "$OUT"/c4_*.log ;;
    kernarg) run kernarg 60 tools/probes/kernarg_probe ;;
    pytestgpu) run pytest_gpu 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
