mkdir -p gpurun_out/r04_s22
B="python bench.py --steps 20 --warmup 5 --window-trace 40 --steady-steps 50000 --extra-blocks= --bridge-steps 0 --config-blocks="
for rep in 1 2; do
  for v in b1 b2 b0 c4; do
    case $v in
      b1) E="" ; X="" ;;
      b2) E="TORCHKAFKA_SPAN_BURST=2" ; X="" ;;
      b0) E="TORCHKAFKA_SPAN_BURST=0" ; X="" ;;
      c4) E="" ; X="--coalesce 4" ;;
    esac
    env $E timeout -k 10 200 $B $X > gpurun_out/r04_s22/$v.$rep.log 2>&1 || exit $?
    echo "$v.$rep done"
  done
done
