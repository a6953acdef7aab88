# round 6, session 21: the HBM mirror's ordering under contention (tools/probes/mirror_stress.hip):
# one process, then four at once (the four-rank rehearsal's load), in the mirror's no-wait mode (0),
# its wait mode (1) and with a plain stream wait per read (2).  Any bad word = a reader saw a buffer
# whose copy was not complete (or was refilled under it).
set -o pipefail
O=gpurun_out/r06_s21
mkdir -p $O
B=tools/probes/bin/mirror_stress
run() {
  local n=$1; shift
  timeout -k 10 120 $B "$@" > $O/$n.json 2> $O/$n.err; local rc=$?
  echo "$n rc=$rc $(cat $O/$n.json) $(head -c 300 $O/$n.err)"
  [ $rc -le 1 ] || exit 1
}
four() {
  local n=$1; shift
  local pids=()
  for k in 1 2 3 4; do timeout -k 10 180 $B "$@" > $O/${n}_$k.json 2> $O/${n}_$k.err & pids+=($!); done
  local worst=0
  for p in "${pids[@]}"; do wait $p; rc=$?; [ $rc -gt $worst ] && worst=$rc; done
  for k in 1 2 3 4; do echo "$n.$k $(cat $O/${n}_$k.json) $(head -c 300 $O/${n}_$k.err)"; done
  [ $worst -le 1 ] || { echo "$n worst rc=$worst"; exit 1; }
}
run m0_p1 1024 8 4 16 0 4
four m0_x4 1024 8 4 16 0 4
four m1_x4 1024 8 4 16 1 4
four m2_x4 1024 8 4 16 2 4
four m0_k8_x4 1024 8 8 16 0 4
# the real loader: the four-rank dma block (the failing one), default / one workgroup per segment /
# the mirror's wait mode, two runs each; a failure is now reported in the line (guarded blocks)
port=0
for v in default parts1 wait; do
  for rep in 1 2; do
    n=dma_${v}_$rep; port=$((port + 1))
    case $v in parts1) export TORCHKAFKA_SPAN_PARTS=1;; wait) export TORCHKAFKA_MIRROR_WAIT=1;; esac
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $((29670 + port)) bench.py --gpus 4 --same-device --steps 20 --warmup 5 --steady-steps 2000 --extra-steps 50000 --extra-blocks dma --config-blocks "" --bridge-steps 0 > $O/$n.json 2> $O/$n.err; rc=$?
    unset TORCHKAFKA_SPAN_PARTS TORCHKAFKA_MIRROR_WAIT
    echo "$n rc=$rc"; [ $rc -eq 0 ] || { grep -E "Error|error" $O/$n.err | head -5; exit 1; }
    python -c "
import json; d = json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
b = d['steady_dma']; print('$n', b.get('error') or (round(b['records_per_s'] / 1e6, 2), b.get('mirror')))"
  done
done
echo session done
