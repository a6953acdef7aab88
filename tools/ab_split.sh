# span decode split over workgroups: GPU tests, then 20-step windows and steady state per split
R=$PWD
O=gpurun_out/r04_s24
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_span_split.py tests/test_gpu_span.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; exit 1; }
tail -2 $O/pytest_split.log
B="python bench.py --steps 20 --warmup 5 --window-trace 40 --steady-steps 50000 --extra-blocks= --bridge-steps 0 --config-blocks="
for rep in 1 2; do
  for sp in 1 2 4; do
    TORCHKAFKA_SPAN_SPLIT=$sp timeout -k 10 200 $B > $O/s$sp.$rep.log 2>&1 || exit $?
    TORCHKAFKA_MIRROR_SPLIT=$sp timeout -k 10 200 $B --h2d dma > $O/m$sp.$rep.log 2>&1 || exit $?
    echo "split $sp rep $rep done"
  done
done
