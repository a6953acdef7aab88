# pipelined span kernels + per-loader command queue: GPU decode tests, sync probe, compute overlap
set -o pipefail
O=gpurun_out/r05_s3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_json_span.py tests/test_gpu_kernels.py tests/test_gpu_loader.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_span.log 2>&1 || { tail -40 $O/pytest_span.log; exit 1; }
tail -3 $O/pytest_span.log
timeout -k 10 120 python tools/probes/sync_probe.py > $O/sync_probe.json 2>&1 || { cat $O/sync_probe.json; exit 1; }
cat $O/sync_probe.json
for v in "config2 zerocopy" "config2 dma" "config4 auto"; do
  set -- $v
  timeout -k 10 300 python benchmarks/compute_overlap.py --workload $1 --h2d $2 > $O/$1_$2.json 2> $O/$1_$2.err || exit $?
  python -c "import json,sys; d=json.load(open('$O/$1_$2.json')); print('$1 $2', d['loader_alone_records_per_s'], d['together']['records_per_s'], d['gemm_alone']['tflops_sum'], d['together']['gemm']['tflops_sum'], d.get('gemm_slowdown_pct'))"
done
