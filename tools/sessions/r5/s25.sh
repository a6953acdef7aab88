# round 5, session 25: the new RCCL-lockstep defaults (normal priority, 64-deep ring, depth 32),
# against steady_state, three runs; the RCCL GPU tests
set -o pipefail
O=gpurun_out/r05_s25
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra-blocks rccl,rccl_sync --config-blocks "" --bridge-steps 0 > $O/b_$i.json 2> $O/b_$i.err; rc=$?
  fatal $rc b$i; [ $rc -eq 0 ] || { tail -5 $O/b_$i.err; exit 1; }
  python - $O/b_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s, r, q = d["steady_state"], d["steady_rccl"], d["steady_rccl_sync"]
print("steady", round(s["records_per_s"] / 1e6, 1), "rccl", round(r["records_per_s"] / 1e6, 1), round(r["records_per_s"] / s["records_per_s"] - 1, 3),
      "wait/step", r.get("lockstep_wait_us_per_step"), "agreements", r.get("lockstep_agreements"), "commit", r.get("commit"), r.get("batches_per_commit"),
      "| sync", round(q["records_per_s"] / 1e6, 2), q["commits"], "p99", r["commit_latency_p99_us"], "ring", r["ring_slots"])
PY
done
timeout -k 10 600 python -u -m pytest tests/test_zz_gpu_rccl.py tests/test_gpu_sync_lockstep.py -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; fatal $rc pytest
echo session done
