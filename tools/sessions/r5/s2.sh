set -o pipefail
O=gpurun_out/r05_s2
mkdir -p $O
export TMPDIR=/tmp
for p in normal high low; do
  TORCHKAFKA_DECODE_PRIORITY=$p timeout -k 10 300 python benchmarks/compute_overlap.py --workload config2 --h2d zerocopy > $O/zc_$p.json 2> $O/zc_$p.err || exit $?
  echo "$p $(cat $O/zc_$p.json)"
done
TORCHKAFKA_DECODE_PRIORITY=high timeout -k 10 300 python benchmarks/compute_overlap.py --workload config2 --h2d dma > $O/dma_high.json 2> $O/dma_high.err || exit $?
echo "dma high $(cat $O/dma_high.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python benchmarks/compute_overlap.py --workload config2 --h2d zerocopy --steps 5000 --gemms 10 > $O/prof.json 2> $O/prof.err || exit $?
echo done
