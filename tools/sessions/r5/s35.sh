# round 5, session 35: why the HBM mirror loses 40 % under the RCCL lockstep -- the dma block with
# the RCCL block's stream layout (2 decode streams, 1 mirror copy stream) but no lockstep, and the
# mirror's fallback counts in both
set -o pipefail
O=gpurun_out/r05_s35
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
run() {  # name, env assignments..., --, bench args
  local n=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config-blocks "" --bridge-steps 0 "$@" > $O/b_$n.json 2> $O/b_$n.err; rc=$?
  fatal $rc $n; [ $rc -eq 0 ] || { tail -5 $O/b_$n.err; exit 1; }
  python3 - $O/b_$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("steady_state", "steady_dma", "steady_rccl"):
    if k in d:
        b = d[k]
        print(sys.argv[2], k, round(b["records_per_s"] / 1e6, 1), b.get("h2d"), b.get("mirror"), "fill", b["worker_fill_us_per_batch"])
PY
}
run base X=1 -- --extra-blocks dma,rccl --h2d dma
run layout TORCHKAFKA_DECODE_STREAMS=2 TORCHKAFKA_MIRROR_COPY_STREAMS=1 -- --extra-blocks dma --h2d dma
run layout_auto TORCHKAFKA_DECODE_STREAMS=2 TORCHKAFKA_MIRROR_COPY_STREAMS=1 -- --extra-blocks dma
echo session done
