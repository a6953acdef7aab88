# round 6, session 3: the teardown / shm tests again, then the same-box A/B and the 2-rank rehearsal
# (session 2's steps after pytest), and the new train_step block alone
set -o pipefail
O=gpurun_out/r06_s3
mkdir -p $O
ROOT=$PWD
timeout -k 10 300 python -u -m pytest tests/test_zz_gpu_rccl.py -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -8 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 1
for wl in "config4 auto"; do
  set -- $wl
  timeout -k 10 200 python benchmarks/train_step.py --workload $1 --h2d $2 > $O/train_$1_$2.json 2> $O/train_$1_$2.err; rc=$?
  echo "train $1 $2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/train_$1_$2.err; exit 1; }
  cat $O/train_$1_$2.json
done
for rep in 1 2; do
  for t in head r4; do
    d=$ROOT; [ $t = r4 ] && d=$ROOT/_ab/r4
    (cd $d && timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --config-blocks "" > $ROOT/$O/drv_${t}_$rep.json 2> $ROOT/$O/drv_${t}_$rep.err); rc=$?
    echo "$t $rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/drv_${t}_$rep.err; exit 1; }
  done
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 2 --same-device --steps 2000 --warmup 200 --extra-blocks shm_sync --config-blocks "" --bridge-steps 0 > $O/two_rank.json 2> $O/two_rank.err; rc=$?
echo "two-rank rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/two_rank.err; exit 1; }
python tools/sessions/r6/summarize.py $O
echo session done
