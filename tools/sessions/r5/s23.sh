# round 5, session 23: the whole GPU suite with HBM segments split over 4 workgroups; the loader
# with parts 1 / 4 (mirror and JSON blocks)
set -o pipefail
O=gpurun_out/r05_s23
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
TORCHKAFKA_SPAN_PARTS=4 timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_parts4.log 2>&1; rc=$?
tail -4 $O/pytest_parts4.log; fatal $rc pytest
for i in 1 2; do
  for p in 1 4; do
    TORCHKAFKA_SPAN_PARTS=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-blocks dma --extra-steps 20000 --config-blocks config4 --config4-steps 20000 --bridge-steps 0 > $O/bench_p${p}_$i.json 2> $O/bench_p${p}_$i.err; rc=$?
    fatal $rc bench$p; [ $rc -eq 0 ] || { tail -5 $O/bench_p${p}_$i.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_p${p}_$i.json').read().strip().splitlines()[-1]); print('parts $p run $i head', round(d['value']/1e6,1), 'steady', round(d['steady_state']['records_per_s']/1e6,1), 'dma', round(d['steady_dma']['records_per_s']/1e6,1), 'config4', round(d['config4']['value']/1e6,1))"
  done
done
echo session done
