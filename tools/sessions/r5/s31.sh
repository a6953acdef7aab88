# round 5, session 31: with the lane-constant merge and 8 parts, the driver's 20-step window and the
# steady state for fixed-width records from the HBM mirror (h2d dma) against zero-copy (the default),
# alternated three times; the RCCL block under each
set -o pipefail
O=gpurun_out/r05_s31
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for i in 1 2 3; do
  for h in auto dma; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --h2d $h --extra-blocks rccl --extra-steps 20000 --config-blocks "" --bridge-steps 0 > $O/b_${h}_$i.json 2> $O/b_${h}_$i.err; rc=$?
    fatal $rc b$h$i; [ $rc -eq 0 ] || { tail -5 $O/b_${h}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${h}_$i.json').read().strip().splitlines()[-1]); s=d['steady_state']['records_per_s']; r=d['steady_rccl']['records_per_s']; print('$h run $i head', round(d['value']/1e6,1), 'steady', round(s/1e6,1), 'rccl', round(r/1e6,1), round(r/s-1,3), d['config']['h2d'])"
  done
done
echo session done
