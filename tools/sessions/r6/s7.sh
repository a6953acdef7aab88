# round 6, session 7: kernel trace of the final tree (steady state, the shm barrier every step,
# the RCCL lockstep at its default cadence), and the RCCL async block with the fitted single
# decode stream against two
set -o pipefail
O=gpurun_out/r06_s7
mkdir -p $O
for ds in fit 2; do
  extra=""; [ $ds = 2 ] && extra="--decode-streams 2"
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 50000 --extra-blocks rccl,shm $extra --config-blocks "" --bridge-steps 0 > $O/rccl_ds$ds.json 2> $O/rccl_ds$ds.err; rc=$?
  echo "rccl ds=$ds rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/rccl_ds$ds.err; exit 1; }
done
python tools/sessions/r6/summarize.py $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 20000 --extra-blocks shm_sync,rccl --config-blocks "" --bridge-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_bench.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $db --md $O/kernels.md > /dev/null && head -12 $O/kernels.md
python tools/probes/lockstep_trace.py $db | tee $O/lockstep_trace.txt
rm -f $db
echo session done
