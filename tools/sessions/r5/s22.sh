# round 5, session 22: device partial CRCs with parts against the host emulation; the mirror tests
set -o pipefail
O=gpurun_out/r05_s22
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for p in 1 2 4; do
  timeout -k 10 120 tools/probes/bin/span_bench_v3 30 128 20 $p > $O/probe_p$p.json 2> $O/probe_p$p.err; rc=$?
  cat $O/probe_p$p.json; fatal $rc probe$p; [ $rc -eq 0 ] || exit 1
done
for p in 2 4; do
  TORCHKAFKA_SPAN_PARTS=$p timeout -k 10 300 python -u -m pytest tests/test_gpu_span.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "mirror_pins_only or growing_log" > $O/pytest_p$p.log 2>&1; rc=$?
  echo "parts $p: $(tail -1 $O/pytest_p$p.log)"; fatal $rc p$p
done
echo session done
