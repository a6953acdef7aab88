# round 5, session 42: VarLen tokens under the RCCL lockstep -- the HBM mirror (auto, two copy
# streams) against the pinned logs, and without the lockstep
set -o pipefail
O=gpurun_out/r05_s42
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
cd benchmarks
for i in 1 2; do
  for v in "off auto" "rccl auto" "rccl zerocopy" "off zerocopy"; do
    set -- $v
    n=$1_$2_$i
    timeout -k 10 300 python varlen_tokens.py --steps 20000 --lockstep $1 --h2d $2 > ../$O/vl_$n.json 2> ../$O/vl_$n.err; rc=$?
    fatal $rc $n; [ $rc -eq 0 ] || { tail -5 ../$O/vl_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('../$O/vl_$n.json').read().strip().splitlines()[-1]); l=d['loader']; print('$n', round(d['value']/1e6,1), d['gb_per_s'], d['lockstep'], d['decode'], 'fallbacks', l.get('mirror_fallbacks'), 'backoffs', l.get('mirror_backoffs'))"
  done
done
echo session done
