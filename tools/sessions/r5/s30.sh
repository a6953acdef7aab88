# round 5, session 30: the lane-constant CRC merge (one multiplication per lane, one returning
# atomic per part) against the shift-table tree -- span_bench v4 (tree) / v5 (lane constants) on
# one box -- then the span / JSON-span GPU tests
set -o pipefail
O=gpurun_out/r05_s30
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for v in v5 v4; do
  for cfg in "16 128 200 1" "16 128 200 4" "16 128 200 8" "16 10 200 1"; do
    n=${v}_$(echo $cfg | tr ' ' '_')
    timeout -k 10 120 tools/probes/bin/span_bench_$v $cfg > $O/sb_$n.json 2> $O/sb_$n.err; rc=$?
    fatal $rc $n; [ $rc -eq 0 ] || { cat $O/sb_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/sb_$n.json')); h=d['hbm']; z=d['pcie_zero_copy']; print('$n', 'pcie', z['lone_us_p50'], z['busy_gb_per_s'], z['verdict'], z['value_mismatches'], '| hbm', h['lone_us_p50'], h['busy_gb_per_s'], h['cu_us_per_mib_upper'], h['verdict'], h['value_mismatches'], '| partials', d['partials'], 'nocrc', d['hbm_nocrc_lone_us_p50'], 'empty', d['empty_lone_us_p50'])"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_span_parts.py tests/test_gpu_json_span.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_span.log 2>&1; rc=$?
tail -3 $O/pytest_span.log; fatal $rc pytest; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_span.log | head -20; exit 1; }
echo session done
