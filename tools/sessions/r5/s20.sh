# round 5, session 20: segments split over 2 / 4 workgroups (SpanLaunch::parts): lone-group latency
# (probe, values + CRC verdict checked), the span / JSON / var-len GPU tests with parts on, and the
# loader's 20-step window and steady state per parts setting
set -o pipefail
O=gpurun_out/r05_s20
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for p in 1 2 4; do
  timeout -k 10 120 tools/probes/bin/span_bench_v3 16 128 200 $p > $O/span_bench_p$p.json 2> $O/span_bench_p$p.err; rc=$?
  cat $O/span_bench_p$p.json; fatal $rc probe$p; [ $rc -eq 0 ] || exit 1
done
for p in 4 2; do
  TORCHKAFKA_SPAN_PARTS=$p timeout -k 10 600 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_json_span.py tests/test_gpu_loader.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_parts$p.log 2>&1; rc=$?
  tail -3 $O/pytest_parts$p.log; fatal $rc pytest$p; [ $rc -eq 0 ] || exit 1
done
for i in 1 2; do
  for p in 1 4 2; do
    TORCHKAFKA_SPAN_PARTS=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-blocks dma --extra-steps 20000 --config-blocks config4 --config4-steps 20000 --bridge-steps 0 > $O/bench_p${p}_$i.json 2> $O/bench_p${p}_$i.err; rc=$?
    fatal $rc bench$p; [ $rc -eq 0 ] || { tail -5 $O/bench_p${p}_$i.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_p${p}_$i.json').read().strip().splitlines()[-1]); print('parts $p run $i head', round(d['value']/1e6,1), 'steady', round(d['steady_state']['records_per_s']/1e6,1), 'dma', round(d['steady_dma']['records_per_s']/1e6,1), 'config4', round(d['config4']['value']/1e6,1))"
  done
done
echo session done
