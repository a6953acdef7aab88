# round 6, session 9: the RCCL async block on the round-5 tree (9560229, built in _ab/head) against
# this tree, alternated, and the bridge blocks with the replica rings' pages faulted in up front
set -o pipefail
O=gpurun_out/r06_s9
mkdir -p $O
ROOT=$PWD
for rep in 1 2; do
  for t in head r5; do
    d=$ROOT; [ $t = r5 ] && d=$ROOT/_ab/head
    (cd $d && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 50000 --extra-blocks rccl --config-blocks "" --bridge-steps 0 > $ROOT/$O/rccl_${t}_$rep.json 2> $ROOT/$O/rccl_${t}_$rep.err); rc=$?
    echo "$t $rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/rccl_${t}_$rep.err; exit 1; }
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra-blocks dma,f32,label --config-blocks "" > $O/bridge_after_blocks.json 2> $O/bridge_after_blocks.err; rc=$?
echo "bridge rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bridge_after_blocks.err; exit 1; }
python tools/sessions/r6/summarize.py $O
python - $O <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/rccl_*.json")):
    b = json.loads(open(f).read().strip().splitlines()[-1])["steady_rccl"]
    print(f.split("/")[-1], {k: b.get(k) for k in ("records_per_s", "ring_slots", "lockstep_agreements", "batches_per_commit", "lockstep_issue_us_per_step", "lockstep_wait_us_per_step", "worker_fill_us_per_batch")}, (b.get("lockstep") or {}).get("streams"))
PY
echo session done
