# round 6, session 12: the JSON parse kernel counting its own row when the width is fixed (pad_to):
# the JSON GPU tests, then config 4 at pad_to 256 with the fused count against the separate count
# kernel (TORCHKAFKA_JSON_FUSED_COUNT=0), alternated, and a kernel trace of each
set -o pipefail
O=gpurun_out/r06_s12
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_json_span.py tests/test_gpu_json_parse.py -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_json.log 2>&1; rc=$?
tail -4 $O/pytest_json.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/pytest_json.log | head -20; exit 1; }
for rep in 1 2; do
  for f in 1 0; do
    n=c4_pad256_fused${f}_$rep
    TORCHKAFKA_JSON_FUSED_COUNT=$f timeout -k 10 200 python benchmarks/config4_json_varlen.py --pad-to 256 > $O/$n.json 2> $O/$n.err; rc=$?
    echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
  done
  n=c4_default_$rep
  timeout -k 10 200 python benchmarks/config4_json_varlen.py > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_s12/c4_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"] / 1e6, 2), "M rec/s", d["gb_per_s_text"], "GB/s", d["last_batch_shape"], d["decode"])
PY
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for f in 1 0; do
  TORCHKAFKA_JSON_FUSED_COUNT=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$f -o run -- python benchmarks/config4_json_varlen.py --steps 4000 --pad-to 256 > $O/prof_c4_fused$f.json 2> $O/prof_c4_fused$f.err; rc=$?
  echo "prof fused=$f rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_c4_fused$f.err; exit 1; }
  db=$(ls $O/prof$f/*/*.db $O/prof$f/*.db 2>/dev/null | head -1)
  python tools/rocpd_summary.py $db --md $O/kernels_c4_fused$f.md > /dev/null && head -8 $O/kernels_c4_fused$f.md
  rm -rf $O/prof$f
done
echo session done
