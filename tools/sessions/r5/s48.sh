# round 5, session 48: coalesce 6 (default) against 8 for the label / unverified / dma blocks
set -o pipefail
O=gpurun_out/r05_s48
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for i in 1 2; do
  for c in 6 8; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --coalesce $c --extra-blocks label,verify,dma --config-blocks "" --bridge-steps 0 > $O/b_c${c}_$i.json 2> $O/b_c${c}_$i.err; rc=$?
    fatal $rc c$c; [ $rc -eq 0 ] || { tail -5 $O/b_c${c}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_c${c}_$i.json').read().strip().splitlines()[-1]); f=lambda k: round(d[k]['records_per_s']/1e6,1); print('coalesce $c run $i head', round(d['value']/1e6,1), 'steady', f('steady_state'), 'label', f('steady_label'), 'unverified', f('steady_unverified'), 'dma', f('steady_dma'))"
  done
done
echo session done
