# round 5, session 45: coalesce 4 / 6 / 8 after the lane-constant merge -- the 20-step window and
# the steady state, alternated
set -o pipefail
O=gpurun_out/r05_s45
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for i in 1 2 3; do
  for c in 8 6 4; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --coalesce $c --extra-blocks "" --config-blocks "" --bridge-steps 0 > $O/b_c${c}_$i.json 2> $O/b_c${c}_$i.err; rc=$?
    fatal $rc c$c; [ $rc -eq 0 ] || { tail -5 $O/b_c${c}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_c${c}_$i.json').read().strip().splitlines()[-1]); print('coalesce $c run $i head', round(d['value']/1e6,1), 'steady', round(d['steady_state']['records_per_s']/1e6,1))"
  done
done
echo session done
