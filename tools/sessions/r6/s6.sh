# round 6, session 6: the JSON count kernel with its framing bytes read from the first loaded pass
# (json_span.hip scan_row): the JSON GPU tests (bit-exact with json.loads / the host scan), then a
# kernel trace of config 4 against session 4's (profiles/r06_s4/kernels_c4.md); the bridge in-flight A/B
set -o pipefail
O=gpurun_out/r06_s6
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_json_span.py tests/test_gpu_json_parse.py -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_json.log 2>&1; rc=$?
tail -4 $O/pytest_json.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python benchmarks/config4_json_varlen.py --steps 4000 > $O/prof_c4.json 2> $O/prof_c4.err; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_c4.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $db --md $O/kernels_c4.md > /dev/null && head -6 $O/kernels_c4.md
rm -f $db
timeout -k 10 300 python benchmarks/config4_json_varlen.py > $O/config4.json 2> $O/config4.err; rc=$?
echo "config4 rc=$rc"; [ $rc -eq 0 ] || exit 1
python -c "import json; d=json.loads(open('$O/config4.json').read().strip().splitlines()[-1]); print({k: d[k] for k in d if 'records_per_s' in k or k in ('decode','h2d')})"
# the bridge's compressed path with 2 / 4 / 8 record sets in flight per partition (the fetch threads
# wait on the inflaters at 2: inflaters 34 % busy, fetch threads 48 % waiting, profiles/r06_s5)
for n in 2 4 8; do
  TORCHKAFKA_BRIDGE_INFLIGHT=$n timeout -k 10 300 python bench.py --steps 20 --warmup 5 --steady-steps 2000 --extra-blocks "" --config-blocks "" --bridge-steps 8000 > $O/bridge_inflight$n.json 2> $O/bridge_inflight$n.err; rc=$?
  echo "bridge inflight $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bridge_inflight$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bridge_inflight$n.json').read().strip().splitlines()[-1])['bridge']; print($n, {k: (round(v['records_per_s']/1e6, 2), v.get('fetch_thread_time_share'), v.get('inflater_time_share')) for k, v in d.items() if isinstance(v, dict)})"
done
echo session done
