#!/bin/bash
# Ad-hoc GPU session: each step under its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 15 "gpurun_out/$name.log"
  echo "=== $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for s in ${STEPS:-pytest_new}; do
  case $s in
    pytest_var) run pytest_var 300 python -u -m pytest tests/test_gpu_span.py -k "var_span" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    pytest_new) run pytest_new 400 python -u -m pytest tests/test_gpu_json_span.py tests/test_gpu_span.py tests/test_gpu_json_parse.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    pytest_all) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    config4) run config4 300 python benchmarks/config4_json_varlen.py ;;
    config4host) run config4_hostdecode 300 python benchmarks/config4_json_varlen.py --decode host ;;
    config4w) for w in 6 8; do run config4_w$w 300 python benchmarks/config4_json_varlen.py --workers $w; done ;;
    config4dma) run config4_dma 300 python benchmarks/config4_json_varlen.py --h2d dma ;;
    bench) run bench 300 python bench.py --stats ;;
    benchdma) run bench_dma 300 python bench.py --stats --h2d dma ;;
    benchdrv) run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    profc4) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/profc4" -o run -- python3 "$OLDPWD/benchmarks/config4_json_varlen.py" --steps 300 > "$OLDPWD/gpurun_out/profc4.log" 2>&1) || exit $?
            tail -5 gpurun_out/profc4.log ;;
    dmasweep) for c in 2 4 16 32; do run bench_dma_c$c 300 python bench.py --stats --h2d dma --mirror-chunk-mib $c --steps 1000; done ;;
    profc4api) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --runtime-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/profc4api" -o run -- python3 "$OLDPWD/benchmarks/config4_json_varlen.py" --steps 2000 > "$OLDPWD/gpurun_out/profc4api.log" 2>&1) || exit $?
            tail -2 gpurun_out/profc4api.log ;;
    profbenchapi) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --runtime-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/profbenchapi" -o run -- python3 "$OLDPWD/bench.py" --steps 2000 --steady-steps 4000 --extra-blocks "" --bridge-steps 0 > "$OLDPWD/gpurun_out/profbenchapi.log" 2>&1) || exit $?
            tail -2 gpurun_out/profbenchapi.log ;;
    profdma) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/profdma" -o run -- python3 "$OLDPWD/bench.py" --h2d dma --steps 1000 --steady-steps 4000 --extra-blocks "" --bridge-steps 0 > "$OLDPWD/gpurun_out/profdma.log" 2>&1) || exit $?
            tail -3 gpurun_out/profdma.log ;;
    config5) run config5 300 python benchmarks/config5_large_messages.py ;;
    config5w) for w in 2 4; do run config5_w$w 300 python benchmarks/config5_large_messages.py --workers $w; done ;;
    bench2r) run bench_2rank_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --same-device --steps 2000 --warmup 200 --stats ;;
    benchf32) run bench_f32 300 python bench.py --stats --dtype f32 ;;
    benchhost) run bench_host 300 python bench.py --stats --decode host ;;
    benchlockr) run bench_lock_rccl 300 python bench.py --lockstep rccl --stats ;;
    profbench) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/profbench" -o run -- python3 "$OLDPWD/bench.py" --steps 1000 --steady-steps 2000 --extra-blocks "" --bridge-steps 0 > "$OLDPWD/gpurun_out/profbench.log" 2>&1) || exit $?
            tail -2 gpurun_out/profbench.log ;;
    pmcspan) (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OLDPWD/gpurun_out/pmc_span" -o run -- python3 "$OLDPWD/bench.py" --steps 200 --warmup 20 --steady-steps 0 --extra-blocks "" --bridge-steps 0 > "$OLDPWD/gpurun_out/pmc_span.log" 2>&1) || exit $?
             tail -2 gpurun_out/pmc_span.log ;;
    pmcjspan) (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OLDPWD/gpurun_out/pmc_jspan" -o run -- python3 "$OLDPWD/benchmarks/config4_json_varlen.py" --steps 200 --warmup 10 > "$OLDPWD/gpurun_out/pmc_jspan.log" 2>&1) || exit $?
             tail -2 gpurun_out/pmc_jspan.log ;;
    pmcfetch) (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$OLDPWD/gpurun_out/pmc_fetch_span" -o run -- python3 "$OLDPWD/bench.py" --steps 200 --warmup 20 --steady-steps 0 --extra-blocks "" --bridge-steps 0 --h2d dma > "$OLDPWD/gpurun_out/pmc_fetch_span.log" 2>&1) || exit $?
             tail -2 gpurun_out/pmc_fetch_span.log ;;
    aheaddrv) for a in 0 1 2 4; do for rep in 1 2; do TORCHKAFKA_AHEAD_DEPTH=$a run bench_drv_ahead${a}_$rep 300 python bench.py --gpus 1 --steps 20 --warmup 5 --steady-steps 0 --extra-blocks "" --bridge-steps 0; done; done ;;
    tokens) run tokens_device 300 python benchmarks/varlen_tokens.py
            run tokens_host 300 python benchmarks/varlen_tokens.py --decode host ;;
    tokenslong) run tokens_long_device 300 python benchmarks/varlen_tokens.py --min-len 2048 --max-len 8192 --batch-size 32 --steps 2000
            run tokens_long_host 300 python benchmarks/varlen_tokens.py --min-len 2048 --max-len 8192 --batch-size 32 --steps 2000 --decode host ;;
    proftok) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/proftok" -o run -- python3 "$OLDPWD/benchmarks/varlen_tokens.py" --steps 500 > "$OLDPWD/gpurun_out/proftok.log" 2>&1) || exit $?
             tail -1 gpurun_out/proftok.log | cut -c1-200 ;;
    bridge) run bridge_e2e 600 python benchmarks/bridge_e2e.py
            run bridge_e2e_1node 600 python benchmarks/bridge_e2e.py --nodes 1
            run bridge_e2e_8node 600 python benchmarks/bridge_e2e.py --nodes 8 --workers 8 ;;
    bridgex) run bridge_ring_long 900 python benchmarks/bridge_e2e.py --records 2000000 --stats
             run bridge_ring_long_8n 900 python benchmarks/bridge_e2e.py --records 2000000 --nodes 8 --workers 8 --stats
             run bridge_linear_long 900 python benchmarks/bridge_e2e.py --records 2000000 --ring-mib 0 --stats ;;
    pytest_bridge) run pytest_bridge 400 python -u -m pytest tests/test_gpu_bridge.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  esac
done
echo "=== done"
