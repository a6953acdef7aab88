# round 5, session 49: rocprofv3 kernel trace of the final tree's default blocks (fixed width with
# 6 batches per launch, HBM mirror block, config 4)
set -o pipefail
O=gpurun_out/r05_s49
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 20000 --extra-blocks dma --config-blocks config4 --config4-steps 20000 --bridge-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_bench.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $db --md $O/kernels.md > /dev/null && head -10 $O/kernels.md
rm -f $db
echo session done
