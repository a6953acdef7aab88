set -o pipefail
O=gpurun_out/r05_s1
mkdir -p $O
for v in "config2 zerocopy" "config2 dma" "config4 auto"; do
  set -- $v
  timeout -k 10 300 python benchmarks/compute_overlap.py --workload $1 --h2d $2 > $O/$1_$2.json 2> $O/$1_$2.err || exit $?
  cat $O/$1_$2.json
done
