# round 5, session 46: coalesce 8 against 6 for JSON (config 4) and var-len tokens, alternated
set -o pipefail
O=gpurun_out/r05_s46
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
cd benchmarks
for i in 1 2; do
  for c in 8 6; do
    timeout -k 10 300 python config4_json_varlen.py --coalesce $c > ../$O/c4_c${c}_$i.json 2> ../$O/c4_c${c}_$i.err; rc=$?
    fatal $rc c4$c; [ $rc -eq 0 ] || { tail -5 ../$O/c4_c${c}_$i.err; exit 1; }
    timeout -k 10 300 python varlen_tokens.py --steps 20000 --coalesce $c > ../$O/vl_c${c}_$i.json 2> ../$O/vl_c${c}_$i.err; rc=$?
    fatal $rc vl$c; [ $rc -eq 0 ] || { tail -5 ../$O/vl_c${c}_$i.err; exit 1; }
    python3 -c "import json; a=json.loads(open('../$O/c4_c${c}_$i.json').read().strip().splitlines()[-1]); b=json.loads(open('../$O/vl_c${c}_$i.json').read().strip().splitlines()[-1]); print('coalesce $c run $i config4', round(a['value']/1e6,1), 'varlen', round(b['value']/1e6,1))"
  done
done
echo session done
