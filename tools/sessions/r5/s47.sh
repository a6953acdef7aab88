# round 5, session 47: coalesce 6 for fixed width -- smoke, the whole GPU suite, the driver's bench command, config 4 under RCCL
set -o pipefail
O=gpurun_out/r05_s47
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
tail -1 $O/smoke.log; fatal $rc smoke; [ $rc -eq 0 ] || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
t0=$(date +%s)
TK_BENCH_WATCHDOG=120 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err; rc=$?
echo "driver-style bench rc=$rc wall=$(( $(date +%s) - t0 )) s"; grep "^\[bench\]" $O/bench_driver.err; fatal $rc driver; [ $rc -eq 0 ] || exit 1
python3 - $O/bench_driver.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["steady_state"]["records_per_s"]
print("value", d["value"], "steady", s, "rccl", d["steady_rccl"]["records_per_s"], round(d["steady_rccl"]["records_per_s"] / s - 1, 3))
print("config4", d["config4"]["value"], "config5", d["config5"]["value"], "config1", d["config1"]["value"])
PY
cd benchmarks && timeout -k 10 300 python config4_json_varlen.py --lockstep rccl > ../$O/c4_rccl.json 2> ../$O/c4_rccl.err; rc=$?; cd ..
fatal $rc c4rccl; [ $rc -eq 0 ] || exit 1
python3 -c "import json; d=json.loads(open('$O/c4_rccl.json').read().strip().splitlines()[-1]); print('config4 under RCCL', d['value'], d['decode'])"
echo session done
