# round 6, session 8: where the RCCL lockstep's async cost comes from at world 1 -- the rccl block
# alone per process (no order effects), polling the agreement's event every 8 steps (default),
# never (round 5), and with an agreement every 32 steps; two runs each
set -o pipefail
O=gpurun_out/r06_s8
mkdir -p $O
run() {  # run <name> <poll every> <extra bench args...>
  local name=$1 poll=$2; shift 2
  TORCHKAFKA_RCCL_POLL_EVERY=$poll timeout -k 10 200 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 50000 --extra-blocks rccl --config-blocks "" --bridge-steps 0 "$@" > $O/$name.json 2> $O/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit 1; }
}
for rep in 1 2; do
  run poll8_$rep 8
  run poll0_$rep 0
  run every32_$rep 8 --lockstep-commit-every 32
done
python tools/sessions/r6/summarize.py $O
echo session done
