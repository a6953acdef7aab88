# round 6, session 1: same-box A/B of the round-4 tree (c4516f4, built in _ab/r4) against HEAD with
# the driver's command (alternated, twice each), then a kernel + HIP API trace of the sync-mode RCCL
# lockstep block alone (where a per-step barrier's 20 us go)
set -o pipefail
O=gpurun_out/r06_s1
mkdir -p $O
ROOT=$PWD
for rep in 1 2; do
  for t in head r4; do
    d=$ROOT; [ $t = r4 ] && d=$ROOT/_ab/r4
    (cd $d && timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --config-blocks "" > $ROOT/$O/drv_${t}_$rep.json 2> $ROOT/$O/drv_${t}_$rep.err); rc=$?
    echo "$t $rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/drv_${t}_$rep.err; exit 1; }
  done
done
cd /tmp && export TMPDIR=/tmp && cd $ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --steady-steps 0 --extra-steps 3000 --extra-blocks rccl_sync --config-blocks "" --bridge-steps 0 > $O/sync_trace.json 2> $O/sync_trace.err; rc=$?
echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/sync_trace.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1); echo "db=$db"
python tools/rocpd_summary.py $db --md $O/kernels.md > /dev/null && head -20 $O/kernels.md
python tools/probes/lockstep_trace.py $db | tee $O/lockstep_trace.txt
echo session done
