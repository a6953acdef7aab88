# the headline's first window step by step; HBM mirror (split 2) against zero-copy
O=gpurun_out/${SESSION:-r04_s25}
mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --window-trace 20 --steady-steps 50000 --extra-blocks= --bridge-steps 0 --config-blocks="
for rep in 1 2 3; do
  timeout -k 10 200 $B > $O/z.$rep.log 2>&1 || exit $?
  TORCHKAFKA_MIRROR_SPLIT=2 timeout -k 10 200 $B --h2d dma > $O/m2.$rep.log 2>&1 || exit $?
  echo "rep $rep done"
done
