# round 5, session 33: HBM mirror under the RCCL lockstep (6-9 streams on 4 hardware queues, session
# 32) -- GPU_MAX_HW_QUEUES=8, and one decode stream, against the loader's layout
set -o pipefail
O=gpurun_out/r05_s33
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
run() {  # name, then env assignments
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --h2d dma --steady-steps 5000 --extra-blocks rccl --extra-steps 20000 --config-blocks "" --bridge-steps 0 > $O/b_$n.json 2> $O/b_$n.err; rc=$?
  fatal $rc $n; [ $rc -eq 0 ] || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1]); s=d['steady_state']['records_per_s']; r=d['steady_rccl']; print('$n steady', round(s/1e6,1), 'rccl', round(r['records_per_s']/1e6,1), 'wait/step', r.get('lockstep_wait_us_per_step'), 'streams', r['lockstep'].get('streams'))"
}
for i in 1 2; do
  run q8_$i GPU_MAX_HW_QUEUES=8
  run q8_m2_$i GPU_MAX_HW_QUEUES=8 TORCHKAFKA_MIRROR_COPY_STREAMS=2
  run d1_$i TORCHKAFKA_DECODE_STREAMS=1
done
echo session done
