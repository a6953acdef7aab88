# stream count vs hardware queues beside a GEMM; kernel trace of the zero-copy overlap
set -o pipefail
O=gpurun_out/r05_s4
mkdir -p $O
export TMPDIR=/tmp
run() {  # name "VAR=v ..." args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python benchmarks/compute_overlap.py "$@" > $O/$name.json 2> $O/$name.err || return $?
  python -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['loader_alone_records_per_s']/1e6,2), round(d['together']['records_per_s']/1e6,2), d['gemm_alone']['tflops_sum'], d['together']['gemm']['tflops_sum'], d.get('gemm_slowdown_pct'))"
}
run dma_d2_c1 "TORCHKAFKA_DECODE_STREAMS=2 TORCHKAFKA_MIRROR_COPY_STREAMS=1" --workload config2 --h2d dma || exit $?
run dma_d1_c1 "TORCHKAFKA_DECODE_STREAMS=1 TORCHKAFKA_MIRROR_COPY_STREAMS=1" --workload config2 --h2d dma || exit $?
run c4_d2_c1 "TORCHKAFKA_DECODE_STREAMS=2 TORCHKAFKA_MIRROR_COPY_STREAMS=1" --workload config4 || exit $?
run zc_d2 "TORCHKAFKA_DECODE_STREAMS=2" --workload config2 --h2d zerocopy || exit $?
run zc_d3 "TORCHKAFKA_DECODE_STREAMS=3" --workload config2 --h2d zerocopy || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_zc -o run -- python benchmarks/compute_overlap.py --workload config2 --h2d zerocopy --steps 8000 --gemms 20 > $O/prof_zc.json 2> $O/prof_zc.err || exit $?
TORCHKAFKA_DECODE_STREAMS=2 TORCHKAFKA_MIRROR_COPY_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dma -o run -- python benchmarks/compute_overlap.py --workload config2 --h2d dma --steps 8000 --gemms 20 > $O/prof_dma.json 2> $O/prof_dma.err || exit $?
echo done
