# kernel traces of --window-trace runs at span burst 1 (default) and 0 (every load in flight)
R=$PWD
mkdir -p gpurun_out/r04_s23
cd /tmp && export TMPDIR=/tmp
for b in 1 0 4; do
  TORCHKAFKA_SPAN_BURST=$b timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04_s23/kt_b$b -o run -- python3 $R/bench.py --steps 20 --warmup 5 --window-trace 40 --steady-steps 0 --extra-blocks= --bridge-steps 0 --config-blocks= > $R/gpurun_out/r04_s23/kt_b$b.log 2>&1 || exit $?
done
