# round 5, session 27: the split-segment GPU tests, the whole GPU suite after the DeviceLoader
# split, smoke, and the bridge blocks alone twice (driver-style runs gave async 42-46 M)
set -o pipefail
O=gpurun_out/r05_s27
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_span_parts.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_parts.log 2>&1; rc=$?
tail -4 $O/pytest_parts.log; fatal $rc parts; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_parts.log | head -20; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
tail -1 $O/smoke.log; fatal $rc smoke; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --steady-steps 2000 --extra-blocks "" --config-blocks "" > $O/bench_bridge_$i.json 2> $O/bench_bridge_$i.err; rc=$?
  grep "^\[bench\]" $O/bench_bridge_$i.err; fatal $rc bridge$i; [ $rc -eq 0 ] || exit 1
done
echo session done
