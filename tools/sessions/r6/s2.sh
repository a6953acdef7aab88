# round 6, session 2: the node-local shared-memory lockstep (shm / shm_sync blocks) beside the RCCL
# ones, its GPU tests, a 2-rank rehearsal on one GPU, and the same-box A/B of the round-4 tree
# (c4516f4 in _ab/r4) against this tree (the session-1 results did not come back)
set -o pipefail
O=gpurun_out/r06_s2
mkdir -p $O
ROOT=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_sync_lockstep.py tests/test_zz_gpu_rccl.py tests/test_gpu_teardown.py -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -12 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for t in head r4; do
    d=$ROOT; [ $t = r4 ] && d=$ROOT/_ab/r4
    (cd $d && timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --config-blocks "" > $ROOT/$O/drv_${t}_$rep.json 2> $ROOT/$O/drv_${t}_$rep.err); rc=$?
    echo "$t $rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/drv_${t}_$rep.err; exit 1; }
  done
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 2 --same-device --steps 2000 --warmup 200 --extra-blocks shm_sync --config-blocks "" --bridge-steps 0 > $O/two_rank.json 2> $O/two_rank.err; rc=$?
echo "two-rank rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/two_rank.err; exit 1; }
python - $O <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    row = {"value": d["value"]}
    for k in ("steady_state", "steady_dma", "steady_label", "steady_shm", "steady_shm_sync", "steady_rccl", "steady_rccl_sync"):
        if isinstance(d.get(k), dict):
            row[k] = round(d[k]["records_per_s"] / 1e6, 2)
            if "batches_per_commit" in d[k]:
                row[k + "_bpc"] = d[k]["batches_per_commit"]
    b = d.get("bridge") or {}
    for k in ("async", "sync", "lz4", "zstd"):
        if isinstance(b.get(k), dict):
            row["bridge_" + k] = round(b[k]["records_per_s"] / 1e6, 2)
    print(f.split("/")[-1], row)
PY
echo session done
