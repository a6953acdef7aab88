# round 5, session 41: after the driver / broker file splits -- smoke and the whole GPU suite; PMC
# passes of the span kernel with the shift-table tree (v4) and the lane-constant merge (v5), 8
# parts; a kernel trace of the default loader (fixed width, HBM mirror, config 4)
set -o pipefail
O=gpurun_out/r05_s41
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
tail -1 $O/smoke.log; fatal $rc smoke; [ $rc -eq 0 ] || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
R=$PWD
cd /tmp && export TMPDIR=/tmp
for v in v4 v5; do
  B=$R/tools/probes/bin/span_bench_$v
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $R/$O/$v/pmc1 -o run -- $B 16 128 20 8 > $R/$O/${v}_pmc1.json 2> $R/$O/${v}_pmc1.err; rc=$?
  echo "$v pmc1 rc=$rc"; [ $rc -eq 0 ] || { tail -3 $R/$O/${v}_pmc1.err; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM --output-format csv -d $R/$O/$v/pmc2 -o run -- $B 16 128 20 8 > $R/$O/${v}_pmc2.json 2> $R/$O/${v}_pmc2.err; rc=$?
  echo "$v pmc2 rc=$rc"; [ $rc -eq 0 ] || { tail -3 $R/$O/${v}_pmc2.err; exit 1; }
done
cd $R
for v in v4 v5; do python tools/prof_summary.py $O/$v $O/${v}_summary > /dev/null && sed -n '/PMC counters/,$p' $O/${v}_summary/SUMMARY.md | head -12; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --steady-steps 5000 --extra-steps 5000 --extra-blocks dma --config-blocks config4 --config4-steps 5000 --bridge-steps 0 > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "prof rc=$rc"; fatal $rc prof; [ $rc -eq 0 ] || { tail -5 $O/prof_bench.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $db --md $O/kernels.md > /dev/null && head -12 $O/kernels.md
rm -f $db
echo session done
