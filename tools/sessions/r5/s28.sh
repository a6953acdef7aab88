# round 5, session 28: eight parts per segment -- the lone-group probe at 1 / 2 / 4 / 8 parts, the
# split-segment tests with 8, the HBM-mirror block with 4 against 8
set -o pipefail
O=gpurun_out/r05_s28
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for p in 1 2 4 8; do
  timeout -k 10 120 tools/probes/bin/span_bench_v4 16 128 200 $p > $O/span_bench_p$p.json 2> $O/span_bench_p$p.err; rc=$?
  cat $O/span_bench_p$p.json; echo; fatal $rc probe$p; [ $rc -eq 0 ] || exit 1
done
timeout -k 10 120 tools/probes/bin/span_bench_v4 30 128 20 8 > $O/probe30_p8.json 2> $O/probe30_p8.err; rc=$?
cat $O/probe30_p8.json; echo; fatal $rc probe30; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_span_parts.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_parts.log 2>&1; rc=$?
tail -3 $O/pytest_parts.log; fatal $rc parts; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_parts.log | head -20; exit 1; }
for i in 1 2; do
  for p in 4 8; do
    TORCHKAFKA_SPAN_PARTS=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-blocks dma --extra-steps 20000 --config-blocks "" --bridge-steps 0 > $O/bench_p${p}_$i.json 2> $O/bench_p${p}_$i.err; rc=$?
    fatal $rc bench$p; [ $rc -eq 0 ] || { tail -5 $O/bench_p${p}_$i.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_p${p}_$i.json').read().strip().splitlines()[-1]); print('parts $p run $i head', round(d['value']/1e6,1), 'steady', round(d['steady_state']['records_per_s']/1e6,1), 'dma', round(d['steady_dma']['records_per_s']/1e6,1))"
  done
done
echo session done
