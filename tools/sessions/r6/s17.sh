# round 6, session 17: a single key column handed out as the [rows] view made at group time (no
# per-batch view + select at delivery): the loader GPU tests, then the driver's fixed-width blocks
# three times (label against steady in the same process)
set -o pipefail
O=gpurun_out/r06_s17
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_loader.py -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
for rep in 1 2 3; do
  n=label_$rep
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-blocks label,f32 --config-blocks "" --bridge-steps 0 > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_s17/label_*.json")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    st, lb, f32 = (j[k]["records_per_s"] / 1e6 for k in ("steady_state", "steady_label", "steady_f32"))
    print(f.split("/")[-1], "steady", round(st, 2), "label", round(lb, 2), "f32", round(f32, 2), "label/steady", round(lb / st, 3))
PY
echo session done
