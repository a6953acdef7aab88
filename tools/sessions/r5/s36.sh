# round 5, session 36: the mirror's back-off (stop copying while the copies are behind the decode)
# -- the mirror under the RCCL lockstep and with one copy stream, config 4, the mirror tests
set -o pipefail
O=gpurun_out/r05_s36
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
run() {  # name, env assignments..., --, bench args
  local n=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --bridge-steps 0 "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?
  fatal $rc $n; [ $rc -eq 0 ] || { tail -5 $O/b_$n.err; exit 1; }
  python3 - $O/b_$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("steady_state", "steady_dma", "steady_rccl"):
    if k in d:
        b = d[k]
        print(sys.argv[2], k, round(b["records_per_s"] / 1e6, 1), b.get("h2d"), b.get("mirror"))
if "config4" in d:
    print(sys.argv[2], "config4", round(d["config4"]["value"] / 1e6, 1))
PY
}
for i in 1 2; do
  run base_$i X=1 -- --extra-blocks dma,rccl --h2d dma --config-blocks config4
  run layout_$i TORCHKAFKA_DECODE_STREAMS=2 TORCHKAFKA_MIRROR_COPY_STREAMS=1 -- --extra-blocks dma --config-blocks ""
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_span.py tests/test_gpu_span_parts.py tests/test_gpu_json_span.py tests/test_gpu_loader.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
echo session done
