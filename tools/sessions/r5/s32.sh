# round 5, session 32: fixed-width records from the HBM mirror under the RCCL lockstep lost 40 %
# (session 31) -- one mirror copy stream (the loader's choice under RCCL) against 2 and 4
set -o pipefail
O=gpurun_out/r05_s32
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for i in 1 2; do
  for m in loader 2 4; do
    if [ $m = loader ]; then unset TORCHKAFKA_MIRROR_COPY_STREAMS; else export TORCHKAFKA_MIRROR_COPY_STREAMS=$m; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --h2d dma --steady-steps 5000 --extra-blocks rccl --extra-steps 20000 --config-blocks "" --bridge-steps 0 > $O/b_${m}_$i.json 2> $O/b_${m}_$i.err; rc=$?
    fatal $rc b$m$i; [ $rc -eq 0 ] || { tail -5 $O/b_${m}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${m}_$i.json').read().strip().splitlines()[-1]); s=d['steady_state']['records_per_s']; r=d['steady_rccl']; print('mirror streams $m run $i steady', round(s/1e6,1), 'rccl', round(r['records_per_s']/1e6,1), 'wait/step', r.get('lockstep_wait_us_per_step'), 'streams', r['lockstep'].get('streams'))"
  done
done
unset TORCHKAFKA_MIRROR_COPY_STREAMS
echo session done
