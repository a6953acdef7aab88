# round 5, session 16: RCCL agreement round trip; coalesce 4 with 8 groups ahead vs coalesce 8
set -o pipefail
O=gpurun_out/r05_s16
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python tools/probes/rccl_rtt.py --iters 1500 > $O/rccl_rtt.json 2> $O/rccl_rtt.err; rc=$?
cat $O/rccl_rtt.json; tail -3 $O/rccl_rtt.err; fatal $rc rtt
for i in 1 2 3; do
  for v in c8 c4d8; do
    if [ $v = c8 ]; then envs=""; c=8; else envs="TORCHKAFKA_AHEAD_DEPTH=8"; c=4; fi
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-blocks "" --config-blocks "" --bridge-steps 0 --coalesce $c > $O/${v}_$i.json 2> $O/${v}_$i.err; rc=$?; fatal $rc $v
    python -c "import json; d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1]); print('$v run $i head', d['value'], 'steady', d['steady_state']['records_per_s'])"
  done
done
echo session done
