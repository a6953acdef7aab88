# round 6, session 23: which mirror configuration holds at four ranks on one GPU (session 21: the
# no-wait policy with 8 workgroups per segment failed its device CRC check in every run; one
# workgroup per segment, or the wait policy, passed).  Four more runs of each, then their N = 1 cost.
set -o pipefail
O=gpurun_out/r06_s23
mkdir -p $O
# the parts merge on RecordBatch-sized segments (config 2's 64 x 1 KiB batches: ~66 KiB, 7 windows
# for 8 workgroups) and shorter ones: parts_stress [launches] [streams] [parts] [sets] [segs] [seg_kib]
for kib in 66 40 12 128; do
  timeout -k 10 120 tools/probes/bin/parts_stress_new 20000 4 8 64 12 $kib > $O/parts_$kib.json 2> $O/parts_$kib.err; rc=$?
  echo "parts_$kib rc=$rc $(cat $O/parts_$kib.json) $(head -c 200 $O/parts_$kib.err)"; [ $rc -le 1 ] || exit 1
done
port=0
for rep in 1 2 3 4; do
  for v in parts1 wait; do
    n=dma_${v}_$rep; port=$((port + 1))
    case $v in parts1) export TORCHKAFKA_SPAN_PARTS=1;; wait) export TORCHKAFKA_MIRROR_WAIT=1;; esac
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $((29680 + port)) bench.py --gpus 4 --same-device --steps 20 --warmup 5 --steady-steps 2000 --extra-steps 50000 --extra-blocks dma --config-blocks "" --bridge-steps 0 > $O/$n.json 2> $O/$n.err; rc=$?
    unset TORCHKAFKA_SPAN_PARTS TORCHKAFKA_MIRROR_WAIT
    echo "$n rc=$rc"; [ $rc -eq 0 ] || { grep -E "Error|error" $O/$n.err | head -5; exit 1; }
    python -c "
import json; d = json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
b = d['steady_dma']; print('$n', b.get('error') or (round(b['records_per_s'] / 1e6, 2), b.get('mirror')))"
  done
done
for rep in 1 2; do
  for v in default parts1 wait; do
    n=one_${v}_$rep
    case $v in parts1) export TORCHKAFKA_SPAN_PARTS=1;; wait) export TORCHKAFKA_MIRROR_WAIT=1;; esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks dma --config-blocks "" --bridge-steps 0 > $O/$n.json 2> $O/$n.err; rc=$?
    unset TORCHKAFKA_SPAN_PARTS TORCHKAFKA_MIRROR_WAIT
    echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/$n.err; exit 1; }
    python -c "
import json; d = json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
b = d['steady_dma']; s = d['steady_state']
print('$n steady', round(s['records_per_s'] / 1e6, 2), 'dma', b.get('error') or (round(b['records_per_s'] / 1e6, 2), b.get('mirror')))"
  done
done
echo session done
