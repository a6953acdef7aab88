# v2 span kernels (loader wave, 4-window ring): lone-group timing, GPU decode tests, compute overlap
set -o pipefail
O=gpurun_out/r05_s7
mkdir -p $O
timeout -k 10 120 tools/probes/bin/span_bench_v2 16 128 200 > $O/span_bench_v2.json || exit $?
timeout -k 10 120 tools/probes/bin/span_bench_v2 24 96 200 >> $O/span_bench_v2.json || exit $?
cat $O/span_bench_v2.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_json_span.py tests/test_gpu_kernels.py tests/test_gpu_loader.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_span.log 2>&1 || { tail -40 $O/pytest_span.log; exit 1; }
tail -1 $O/pytest_span.log
run() {  # name "VAR=v ..." args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python benchmarks/compute_overlap.py "$@" > $O/$name.json 2> $O/$name.err || return $?
  python -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['loader_alone_records_per_s']/1e6,2), round(d['together']['records_per_s']/1e6,2), d['gemm_alone']['tflops_sum'], d['together']['gemm']['tflops_sum'], d.get('gemm_slowdown_pct'))"
}
run zc "" --workload config2 --h2d zerocopy || exit $?
run dma "" --workload config2 --h2d dma || exit $?
run c4 "" --workload config4 || exit $?
