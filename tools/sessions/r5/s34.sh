# round 5, session 34: HBM mirror under the RCCL lockstep -- the deep layout (64-slot ring per
# worker, agreements 32 steps ahead) against the shallow one (16 slots, 2 steps), zero-copy beside
set -o pipefail
O=gpurun_out/r05_s34
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --extra-blocks rccl --config-blocks "" --bridge-steps 0 "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?
  fatal $rc $n; [ $rc -eq 0 ] || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1]); s=d['steady_state']['records_per_s']; r=d['steady_rccl']; print('$n steady', round(s/1e6,1), 'rccl', round(r['records_per_s']/1e6,1), round(r['records_per_s']/s-1,3), 'wait/step', r.get('lockstep_wait_us_per_step'), 'agreements', r['lockstep_agreements'], 'fill', r['worker_fill_us_per_batch'], 'slots', r['ring_slots'])"
}
for i in 1 2; do
  run dma_deep_$i --h2d dma
  run dma_shallow_$i --h2d dma --lockstep-depth 2 --slots-per-worker 16
  run dma_mid_$i --h2d dma --lockstep-depth 8 --slots-per-worker 16
done
echo session done
