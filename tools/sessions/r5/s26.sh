# round 5, session 26: final defaults -- smoke, the whole GPU suite, the driver's bench command
# (timed), a kernel trace of the default blocks
set -o pipefail
O=gpurun_out/r05_s26
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log; fatal $rc smoke; [ $rc -eq 0 ] || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; fatal $rc pytest
t0=$(date +%s)
TK_BENCH_WATCHDOG=120 timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err; rc=$?
echo "driver-style bench rc=$rc wall=$(( $(date +%s) - t0 )) s"; grep "^\[bench\]" $O/bench_driver.err; fatal $rc driver
python - $O/bench_driver.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "steady", d["steady_state"]["records_per_s"])
for k in ("steady_dma", "steady_f32", "steady_label", "steady_rccl", "steady_rccl_sync", "steady_unverified"):
    if k in d: print(k, d[k]["records_per_s"], d[k].get("commit"), d[k].get("batches_per_commit"))
for k, v in (d.get("bridge") or {}).items():
    if isinstance(v, dict): print("bridge", k, v["records_per_s"], v.get("gb_per_s"))
for k in ("steady_compute", "config4", "config5", "config1", "process_override"):
    if k in d: print(k, json.dumps(d[k])[:400])
PY
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --steady-steps 5000 --extra-steps 5000 --extra-blocks dma,rccl --config-blocks config4 --config4-steps 5000 --bridge-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "prof rc=$rc"; fatal $rc prof; [ $rc -eq 0 ] || { tail -5 $O/prof_bench.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1); echo "db=$db"
python tools/rocpd_summary.py $db --md $O/kernels.md > /dev/null && head -30 $O/kernels.md
ls $O/prof/*/ $O/prof 2>/dev/null | head
echo session done
