# round 6, session 34: workers map a ring replica whole at its first read (consumer.cpp prefault), on top of
# session 28's whole-ring pinning --
# the bridge GPU tests, then the codec census twice
set -o pipefail
O=gpurun_out/r06_s34
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bridge.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_bridge.log 2>&1; rc=$?
tail -2 $O/pytest_bridge.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_bridge.log | head; exit 1; }
for rep in 1 2; do
  n=codecs_$rep
  TK_BENCH_CPU=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks "" --config-blocks "" --bridge-codecs lz4,zstd > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
  python - "$O/$n.json" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, b in (j.get("bridge") or {}).items():
    if isinstance(b, dict) and "records_per_s" in b:
        c = b.get("cpu", {})
        print(k, round(b["records_per_s"] / 1e6, 2), "fill", b.get("worker_fill_us_per_batch"), json.dumps(c.get("by_name"))[:300])
PY
done
echo session done
