# round 6, session 20: the device CRC failure of session 18's four-rank rehearsal (h2d='dma' block,
# the only path whose launches split a segment over 8 workgroups that merge their CRC partials in an
# accumulator word).  tools/probes/parts_stress.hip: every launch its own verdict word over a log whose
# CRCs are all correct; `old` = the kernel before this session (plain store zeroing the word after
# the merge), `new` = the word zeroed with an agent-scope atomic.  One process, then four at once
# (four ranks on one GPU).  Then the four-rank dma block with the rebuilt extension, twice.
set -o pipefail
O=gpurun_out/r06_s20
mkdir -p $O
B=tools/probes/bin
run() {  # name, binary, args...
  local n=$1; shift
  timeout -k 10 120 "$@" > $O/$n.json 2> $O/$n.err; local rc=$?
  echo "$n rc=$rc $(cat $O/$n.json)"
  [ $rc -le 1 ] || exit 1   # 1 = bad verdicts found (a result), anything else ends the session
}
four() {  # name, binary, args...: four processes at once
  local n=$1; shift
  local pids=()
  for k in 1 2 3 4; do
    timeout -k 10 180 "$@" > $O/${n}_$k.json 2> $O/${n}_$k.err & pids+=($!)
  done
  local worst=0
  for p in "${pids[@]}"; do wait $p; rc=$?; [ $rc -gt $worst ] && worst=$rc; done
  for k in 1 2 3 4; do echo "$n.$k $(cat $O/${n}_$k.json)"; done
  [ $worst -le 1 ] || { echo "$n worst rc=$worst"; exit 1; }
}
# calibration: one set per stream is the round-5 bug (launches on one stream sharing the words)
run old_sets1 $B/parts_stress_old 20000 4 8 1
run old_p1 $B/parts_stress_old 20000 4 8 16
four old_x4 $B/parts_stress_old 20000 4 8 16
four new_x4 $B/parts_stress_new 20000 4 8 16
four new64_x4 $B/parts_stress_new 20000 4 8 64
run new_sets1 $B/parts_stress_new 20000 4 8 1
for rep in 1 2; do
  n=four_dma_$rep
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 2966$rep bench.py --gpus 4 --same-device --steps 20 --warmup 5 --extra-blocks dma --config-blocks "" --bridge-steps 0 > $O/$n.json 2> $O/$n.err; rc=$?
  grep "^\[bench\]" $O/$n.err | tail -5; echo "$n rc=$rc"
  [ $rc -eq 0 ] || { grep -E "Error|error" $O/$n.err | head -5; exit 1; }
  python -c "
import json; d = json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
b = d['steady_dma']; print('$n dma', round(b['records_per_s'] / 1e6, 2), 'M', b.get('mirror'))"
done
echo session done
