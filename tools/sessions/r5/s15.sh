# round 5, session 15: RCCL agreement round trip (idle / beside load / beside a live loader);
# coalesce 8 vs 4 on the 20-step window and the steady state, alternated
set -o pipefail
O=gpurun_out/r05_s15
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python tools/probes/rccl_rtt.py --iters 1500 > $O/rccl_rtt.json 2> $O/rccl_rtt.err; rc=$?
cat $O/rccl_rtt.json; fatal $rc rtt
for i in 1 2 3; do
  for c in 8 4; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-blocks "" --config-blocks "" --bridge-steps 0 --coalesce $c > $O/c${c}_$i.json 2> $O/c${c}_$i.err; rc=$?; fatal $rc c$c
    python -c "import json; d=json.loads(open('$O/c${c}_$i.json').read().strip().splitlines()[-1]); print('coalesce $c run $i head', d['value'], 'steady', d['steady_state']['records_per_s'])"
  done
done
echo session done
