# round 5, session 38: JSON (config 4) under the RCCL lockstep -- the HBM mirror (h2d dma) against
# the pinned logs (h2d auto under RCCL since this session), and without the lockstep
set -o pipefail
O=gpurun_out/r05_s38
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
cd benchmarks
for i in 1 2; do
  for v in "off auto" "rccl auto" "rccl dma" "off zerocopy"; do
    set -- $v
    n=$1_$2_$i
    timeout -k 10 300 python config4_json_varlen.py --lockstep $1 --h2d $2 > ../$O/c4_$n.json 2> ../$O/c4_$n.err; rc=$?
    fatal $rc $n; [ $rc -eq 0 ] || { tail -5 ../$O/c4_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('../$O/c4_$n.json').read().strip().splitlines()[-1]); l=d['loader']; print('$n', round(d['value']/1e6,1), d['lockstep'], d['decode'], 'fallbacks', l.get('mirror_fallbacks'), l.get('mirror_pending_fallbacks'), 'backoffs', l.get('mirror_backoffs'))"
  done
done
echo session done
