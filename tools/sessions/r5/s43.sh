# round 5, session 43: h2d='auto' mirrors JSON rows only (var-len back to zero-copy) -- the span,
# split-segment, JSON, loader and serialized GPU tests; var-len tokens with and without the lockstep
set -o pipefail
O=gpurun_out/r05_s43
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_span_parts.py tests/test_gpu_json_span.py tests/test_gpu_loader.py tests/test_gpu_serialized.py -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
cd benchmarks
for v in off rccl off rccl; do
  timeout -k 10 300 python varlen_tokens.py --steps 20000 --lockstep $v > ../$O/vl_$v.json 2> ../$O/vl_$v.err; rc=$?
  fatal $rc $v; [ $rc -eq 0 ] || { tail -5 ../$O/vl_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('../$O/vl_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), d['gb_per_s'], d['lockstep'], d['decode'])"
done
echo session done
