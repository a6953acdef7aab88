# round 5, session 50: the bench's N > 1 path rehearsed on one GPU -- 2 and 4 ranks on cuda:0 with a
# gloo group (host lockstep), the final tree
set -o pipefail
O=gpurun_out/r05_s50
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for n in 2 4; do
  timeout -k 10 400 python bench.py --gpus $n --same-device --self-launch --steps 20 --warmup 5 --steady-steps 5000 --extra-blocks "" --config-blocks "" --bridge-steps 0 > $O/b_n$n.json 2> $O/b_n$n.err; rc=$?
  fatal $rc n$n; [ $rc -eq 0 ] || { tail -8 $O/b_n$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_n$n.json').read().strip().splitlines()[-1]); print('n $n', d['n_gpus'], d['config']['parallelism'], round(d['value']/1e6,1), round(d['steady_state']['records_per_s']/1e6,1), d['lockstep'], d['per_rank_records_per_s'])"
done
echo session done
