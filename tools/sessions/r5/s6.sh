# span_bench under rocprofv3: kernel time alone, then PMC passes (one per block budget)
set -o pipefail
O=gpurun_out/r05_s6
mkdir -p $O
export TMPDIR=/tmp
B=tools/probes/bin/${SPAN_BENCH:-span_bench_v1}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $B 16 128 50 > $O/kt.json 2> $O/kt.err || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/pmc1 -o run -- $B 16 128 20 > $O/pmc1.json 2> $O/pmc1.err || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM -d $O/pmc2 -o run -- $B 16 128 20 > $O/pmc2.json 2> $O/pmc2.err || exit $?
echo done
