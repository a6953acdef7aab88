# round 5, session 40: the bridge block after the other steady blocks gave 38-46 M against 50 M
# alone -- deferred releases of the earlier loaders running beside it? TORCHKAFKA_DEFERRED_FREE=0
set -o pipefail
O=gpurun_out/r05_s40
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for i in 1 2; do
  for df in 1 0; do
    TORCHKAFKA_DEFERRED_FREE=$df timeout -k 10 400 python bench.py --steps 20 --warmup 5 --extra-blocks dma,f32,label,rccl --config-blocks "" --bridge-codecs "" > $O/b_df${df}_$i.json 2> $O/b_df${df}_$i.err; rc=$?
    fatal $rc df$df; [ $rc -eq 0 ] || { tail -5 $O/b_df${df}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_df${df}_$i.json').read().strip().splitlines()[-1]); b=d['bridge']; print('deferred $df run $i', 'steady', round(d['steady_state']['records_per_s']/1e6,1), 'label', round(d['steady_label']['records_per_s']/1e6,1), 'rccl', round(d['steady_rccl']['records_per_s']/1e6,1), 'bridge', round(b['async']['records_per_s']/1e6,1), round(b['sync']['records_per_s']/1e6,1), 'fill', b['async']['worker_fill_us_per_batch'])"
  done
done
echo session done
