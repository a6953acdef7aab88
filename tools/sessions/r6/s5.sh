# round 6, session 5: the whole GPU suite, then the driver's command with every default block
# (train, compute, config 4/5/1, process, the bridge blocks with the producer timing and lz4_static)
set -o pipefail
O=gpurun_out/r06_s5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err; rc=$?
grep "^\[bench\]" $O/driver.err | tail -40; echo "driver rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/driver.err; exit 1; }
python tools/sessions/r6/summarize.py $O
echo session done
