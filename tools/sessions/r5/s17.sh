# round 5, session 17: kernel trace of the RCCL-lockstep block
set -o pipefail
O=gpurun_out/r05_s17
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --steady-steps 2000 --extra-steps 20000 --extra-blocks rccl --config-blocks "" --bridge-steps 0 > $O/bench.json 2> $O/bench.err; rc=$?
echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1); echo "db=$db"
python tools/probes/lockstep_trace.py $db | tee $O/lockstep_trace.txt
python tools/rocpd_summary.py $db --md $O/kernels.md > /dev/null && head -30 $O/kernels.md
ls -la $db

timeout -k 10 400 python bench.py --steps 20 --warmup 5 --steady-steps 2000 --extra-blocks "" --config-blocks "" > $O/bench_bridge.json 2> $O/bench_bridge.err; rc=$?
grep "^\[bench\]" $O/bench_bridge.err; [ $rc -eq 0 ] || exit 1
python - $O/bench_bridge.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d["bridge"].items():
    if isinstance(v, dict):
        print(k, {x: v[x] for x in v if x in ("records_per_s", "gb_per_s", "wire_gb_per_s", "inflated_batches_in_timed_region", "fetch_threads", "inflate_threads", "inflate_gb_per_s_per_thread", "fetch_thread_time_share", "inflater_time_share", "bridge_errors")})
PY
echo session done
