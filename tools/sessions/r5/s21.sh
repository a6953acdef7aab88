# round 5, session 21: the mirror test that failed with parts = 4 -- with parts 1, 2, 4
set -o pipefail
O=gpurun_out/r05_s21
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for p in 1 2 4; do
  TORCHKAFKA_SPAN_PARTS=$p timeout -k 10 300 python -u -m pytest tests/test_gpu_span.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "mirror_pins_only or growing_log or big" > $O/pytest_p$p.log 2>&1; rc=$?
  echo "parts $p: $(tail -1 $O/pytest_p$p.log)"; fatal $rc p$p
done
echo session done
