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
    pytestloader) step pytest_loader 300 python -u -m pytest tests/test_gpu_loader.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    pytestjson) step pytest_json 300 python -u -m pytest tests/test_gpu_json_parse.py tests/test_gpu_loader.py -k json -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    config4zc) step config4_zc 300 python benchmarks/config4_json_varlen.py --h2d zerocopy ;;
    config4w8) step config4_w8 300 python benchmarks/config4_json_varlen.py --workers 8 ;;
    config4w6) step config4_w6 300 python benchmarks/config4_json_varlen.py --workers 6 ;;
    pmcjson) (cd /tmp && export TMPDIR=/tmp && step pmc_json 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_json" -o run -- python3 "$OLDPWD/benchmarks/config4_json_varlen.py" --steps 100 --warmup 10) || exit $? ;;
    config4s8) step config4_s8 300 python benchmarks/config4_json_varlen.py --slots-per-worker 8 ;;
    config4e1) step config4_e1 300 python benchmarks/config4_json_varlen.py --event-every 1 ;;
    config4s8e1) step config4_s8e1 300 python benchmarks/config4_json_varlen.py --slots-per-worker 8 --event-every 1 ;;
    config4p0) step config4_p0 300 python benchmarks/config4_json_varlen.py --prefetch 0 --event-every 1 ;;
    config4nofence) TORCHKAFKA_EXP_NO_PARSE_FENCE=1 step config4_nofence 300 python benchmarks/config4_json_varlen.py ;;
    config4host) step config4_host 300 python benchmarks/config4_json_varlen.py --json-parse host ;;
    pytest) step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    nccl)   step nccl_probe 120 python tools/nccl_probe.py ;;
    overhead) step host_overhead 120 python tools/host_overhead.py ;;
    lockcheck5) TORCHKAFKA_DRIVER_TRACE=1 LOCKCHECK_DEPTHS=5 step lockstep_check5 150 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29632 tools/lockstep_check.py ;;
    lockrccl) LOCKCHECK_TRANSPORT=rccl LOCKCHECK_DEPTHS=0,3 step lockstep_rccl 120 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29633 tools/lockstep_check.py ;;
    lockjson) LOCKCHECK_SCHEMA=json LOCKCHECK_DEPTHS=0,3 step lockstep_json 150 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29634 tools/lockstep_check.py ;;
    lockcheck) step lockstep_check 150 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 tools/lockstep_check.py ;;
    bench)  step bench 600 python bench.py --stats ;;
    benchlockr) step bench_lock_rccl 600 python bench.py --lockstep rccl --stats ;;
    benchlockoff) step bench_lock_off 600 python bench.py --lockstep off --stats ;;
    bench2r) step bench_2rank_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --same-device --steps 2000 --warmup 200 --stats ;;
    benchdriver) step bench_driver 300 python bench.py --steps 20 --warmup 5 ;;
    pytestspan) step pytest_span 300 python -u -m pytest tests/test_gpu_span.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    spannocrc) step bench_span_nocrc 300 python bench.py --steps 1000 --steady-steps 4000 --no-crc --stats ;;
    spanb1) for n in 2 3 4; do TORCHKAFKA_SPAN_BURST=1 TORCHKAFKA_DECODE_STREAMS=$n step bench_b1s$n 300 python bench.py --steps 1000 --stats; done
            TORCHKAFKA_SPAN_BURST=2 step bench_b2s2 300 python bench.py --steps 1000 --stats
            TORCHKAFKA_SPAN_BURST=1 step bench_b1s2c16 300 python bench.py --steps 1000 --stats --slots-per-worker 32 ;;
    spanburst) for b in 1 2 4 8; do TORCHKAFKA_SPAN_BURST=$b step bench_burst$b 300 python bench.py --steps 1000 --steady-steps 4000; done ;;
    tlbprobe) step tlb_probe 300 tools/probes/bin/tlb_probe ;;
    spanstreams) for n in 1 3 4; do TORCHKAFKA_DECODE_STREAMS=$n step bench_ds$n 300 python bench.py --steps 1000 --stats; done ;;
    ahead) for n in 0 3 4 6; do TORCHKAFKA_AHEAD_DEPTH=$n step bench_ahead$n 300 python bench.py --steps 1000 --stats; done
           TORCHKAFKA_AHEAD_DEPTH=4 step bench_drv_ahead4 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    spanreg) TORCHKAFKA_SPAN_BURST=-1 step bench_spanreg 300 python bench.py --steps 1000 --stats ;;
    spansweep) step sw_s32 300 python bench.py --steps 1000 --slots-per-worker 32 --stats
               step sw_c4 300 python bench.py --steps 1000 --coalesce 4 --stats
               step sw_w6 300 python bench.py --steps 1000 --workers 6 --stats
               step sw_cw0 300 python bench.py --steps 1000 --coalesce-wait-us 0 --stats
               step sw_cw200 300 python bench.py --steps 1000 --coalesce-wait-us 200 --stats
               step sw_pf8 300 python bench.py --steps 1000 --prefetch 8 --stats ;;
    benchhost) step bench_host 600 python bench.py --stats --decode host ;;
    benchdrv) step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    benchf32) step bench_f32 600 python bench.py --stats --dtype f32 ;;
    benchdma2) step bench_dma 600 python bench.py --stats --h2d dma ;;
    bench8) step bench_fp8 600 python bench.py --stats --dtype fp8 ;;
    benchlong) step bench_long 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchnonuma) step bench_nonuma 600 python bench.py --stats --steps 4000 --warmup 100 --no-numa ;;
    benchc1) step bench_c1 600 python bench.py --stats --steps 4000 --warmup 100 --coalesce 1 ;;
    benchc8) step bench_c8 600 python bench.py --stats --steps 4000 --warmup 100 --coalesce 8 ;;
    benchw8c8) step bench_w8c8 600 python bench.py --stats --steps 4000 --warmup 100 --coalesce 8 --workers 8 ;;
    benchdirect) step bench_direct 600 python bench.py --stats --steps 4000 --warmup 100 --h2d direct ;;
    benchdirectc8) step bench_direct_c8 600 python bench.py --stats --steps 4000 --warmup 100 --h2d direct --coalesce 8 ;;
    benchdirectw8) step bench_direct_w8 600 python bench.py --stats --steps 4000 --warmup 100 --h2d direct --workers 8 ;;
    pytestdirect) step pytest_direct 300 python -u -m pytest tests/test_gpu_loader.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "direct" ;;
    benchnospin) TORCHKAFKA_WORKER_SPIN_US=0 step bench_nospin 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchpf0) TORCHKAFKA_CRC_PREFETCH=0 step bench_pf0 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchpf2k) TORCHKAFKA_CRC_PREFETCH=2048 step bench_pf2k 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchpf4k) TORCHKAFKA_CRC_PREFETCH=4096 step bench_pf4k 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchs8) step bench_s8 600 python bench.py --stats --steps 4000 --warmup 100 --slots-per-worker 8 ;;
    benchs8nocrc) step bench_s8nocrc 600 python bench.py --stats --steps 4000 --warmup 100 --slots-per-worker 8 --no-crc ;;
    benchs16) step bench_s16 600 python bench.py --stats --steps 4000 --warmup 100 --slots-per-worker 16 ;;
    benchdmas8) step bench_dma_s8 600 python bench.py --stats --steps 4000 --warmup 100 --slots-per-worker 8 --h2d dma ;;
    benchdmas8c1) step bench_dma_s8c1 600 python bench.py --stats --steps 4000 --warmup 100 --slots-per-worker 8 --h2d dma --coalesce 1 ;;
    profs8) (cd /tmp && export TMPDIR=/tmp && step profs8 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/profs8" -o run -- python3 "$OLDPWD/bench.py" --steps 2000 --stats --slots-per-worker 8) || exit $? ;;
    benchw0) step bench_w0 600 python bench.py --stats --steps 4000 --warmup 100 --coalesce-wait-us 0 ;;
    benchc8w) step bench_c8w 600 python bench.py --stats --steps 4000 --warmup 100 --coalesce 8 ;;
    benchc8w200) step bench_c8w200 600 python bench.py --stats --steps 4000 --warmup 100 --coalesce 8 --coalesce-wait-us 200 ;;
    benchnofold) TORCHKAFKA_CRC_FOLD=0 step bench_nofold 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    fillbench) step fill_bench 300 python tools/fill_bench.py ;;
    fillbenchnofold) TORCHKAFKA_CRC_FOLD=0 step fill_bench_nofold 300 python tools/fill_bench.py ;;
    benchfp2k) TORCHKAFKA_CRC_FOLD_PREFETCH=2048 step bench_fp2k 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchfp4k) TORCHKAFKA_CRC_FOLD_PREFETCH=4096 step bench_fp4k 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchfp512) TORCHKAFKA_CRC_FOLD_PREFETCH=512 step bench_fp512 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchfp8k) TORCHKAFKA_CRC_FOLD_PREFETCH=8192 step bench_fp8k 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchfp16k) TORCHKAFKA_CRC_FOLD_PREFETCH=16384 step bench_fp16k 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchw100) step bench_w100 600 python bench.py --stats --steps 4000 --warmup 100 --coalesce-wait-us 100 ;;
    benchpf4) step bench_pf4 600 python bench.py --stats --steps 4000 --warmup 100 --prefetch 4 ;;
    benchnocrc) step bench_nocrc 600 python bench.py --stats --steps 4000 --warmup 100 --no-crc ;;
    benchzc) step bench_zc 600 python bench.py --stats --steps 4000 --warmup 100 --h2d zerocopy ;;
    benchs1) step bench_s1 600 python bench.py --stats --steps 4000 --warmup 100 --copy-streams 1 ;;
    benchw8) step bench_w8 600 python bench.py --stats --steps 4000 --warmup 100 --workers 8 ;;
    benchnont) TORCHKAFKA_NT_COPY=0 step bench_nont 600 python bench.py --stats --steps 4000 --warmup 100 ;;
    benchee1) step bench_ee1 600 python bench.py --stats --steps 4000 --warmup 100 --event-every 1 ;;
    benchee4) step bench_ee4 600 python bench.py --stats --steps 4000 --warmup 100 --event-every 4 ;;
    benchdma) step bench_dma 600 python bench.py --stats --steps 4000 --warmup 100 --h2d dma ;;
    benchbs) step bench_bs1024 600 python bench.py --stats --steps 2000 --warmup 100 --batch-size 1024 ;;
    config1) step config1 300 python benchmarks/config1_cpu_plumbing.py ;;
    config4) step config4 300 python benchmarks/config4_json_varlen.py ;;
    config5) step config5 300 python benchmarks/config5_large_messages.py ;;
    config5direct) step config5_direct 300 python benchmarks/config5_large_messages.py --h2d direct ;;
    config5w8) step config5_w8 300 python benchmarks/config5_large_messages.py --workers 8 ;;
    example3) step example3 300 python examples/03_device_loader_training.py ;;
    example4) step example4 300 python examples/04_json_device_parse.py ;;
    kbench) step kernel_bench 300 python tools/kernel_bench.py ;;
    kprof)  (cd /tmp && export TMPDIR=/tmp && step kprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kprof" -o run -- python3 "$OLDPWD/tools/kernel_bench.py" --quick) || exit $? ;;
    # TCC has 4 slots per pass: FETCH_SIZE costs 3, WRITE_SIZE 2 (MI355X_MICROARCH.md) -> two passes
    pmc)    (cd /tmp && export TMPDIR=/tmp && step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$OLDPWD/tools/kernel_bench.py" --quick) || exit $?
            (cd /tmp && export TMPDIR=/tmp && step pmc_write 300 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$OLDPWD/tools/kernel_bench.py" --quick) || exit $? ;;
    profcopy) (cd /tmp && export TMPDIR=/tmp && step profcopy 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/profcopy" -o run -- python3 "$OLDPWD/bench.py" --steps 1000) || exit $? ;;
    profnocrc) (cd /tmp && export TMPDIR=/tmp && step profnocrc 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profnocrc" -o run -- python3 "$OLDPWD/bench.py" --steps 2000 --no-crc --stats) || exit $? ;;
    proflong) (cd /tmp && export TMPDIR=/tmp && step proflong 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/proflong" -o run -- python3 "$OLDPWD/bench.py" --steps 2000 --stats) || exit $? ;;
    profc4t) (cd /tmp && export TMPDIR=/tmp && step profc4t 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/profc4t" -o run -- python3 "$OLDPWD/benchmarks/config4_json_varlen.py" --steps 300) || exit $? ;;
    profc4) (cd /tmp && export TMPDIR=/tmp && step profc4 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/profc4" -o run -- python3 "$OLDPWD/benchmarks/config4_json_varlen.py" --steps 300) || exit $? ;;
    profspan) (cd /tmp && export TMPDIR=/tmp && step profspan 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profspan" -o run -- python3 "$OLDPWD/bench.py" --steps 500 --steady-steps 1000 --stats) || exit $? ;;
    prof)   (cd /tmp && export TMPDIR=/tmp && step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$OLDPWD/bench.py" --steps 200) || exit $? ;;
  esac
done
echo "=== done"
