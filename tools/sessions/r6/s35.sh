# round 6, session 35: final validation after the workers map ring replicas whole -- the whole GPU suite, smoke, the
# driver's 1-GPU command with every default block, the driver's N = 4 command rehearsed as four
# ranks sharing this one GPU (every default block but RCCL's), and a kernel trace of the steady state
set -o pipefail
O=gpurun_out/r06_s35
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err; rc=$?
grep "^\[bench\]" $O/driver.err | tail -40 > $O/driver_progress.txt; echo "driver rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/driver.err; exit 1; }
python tools/sessions/r6/summarize.py $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29653 bench.py --gpus 4 --same-device --steps 20 --warmup 5 > $O/four_rank.json 2> $O/four_rank.err; rc=$?
grep "^\[bench\]" $O/four_rank.err | tail -30 > $O/four_rank_progress.txt; echo "four-rank rc=$rc"; [ $rc -eq 0 ] || { tail -8 $O/four_rank.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_s35/four_rank.json").read().strip().splitlines()[-1])
out = {k: d[k] for k in ("metric", "value", "n_gpus", "ms_per_step", "config") if k in d}
for k, v in d.items():
    if isinstance(v, dict) and "records_per_s" in v:
        out[k] = (round(v["records_per_s"] / 1e6, 2), v.get("batches_per_commit"), v.get("per_rank_records_per_s"))
print(json.dumps(out)[:3000])
PY
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 20000 --extra-blocks shm_sync --config-blocks "" --bridge-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_bench.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $db --md $O/kernels.md > /dev/null && head -10 $O/kernels.md
rm -rf $O/prof
echo session done
