# round 6, session 24: the mirror policy change (fixed-width decode: a waiting mirror, segments split
# only under it; JSON / var-len: no-wait, one workgroup per segment) -- the whole GPU suite, the
# four-rank dma block three times (default settings), the driver's 1-GPU command.
set -o pipefail
O=gpurun_out/r06_s24
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
for rep in 1 2 3; do
  n=four_dma_$rep
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $((29690 + rep)) bench.py --gpus 4 --same-device --steps 20 --warmup 5 --steady-steps 2000 --extra-steps 50000 --extra-blocks dma --config-blocks "" --bridge-steps 0 > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc"; [ $rc -eq 0 ] || { grep -E "Error|error" $O/$n.err | head -5; exit 1; }
  python -c "
import json; d = json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
b = d['steady_dma']; print('$n', b.get('error') or (round(b['records_per_s'] / 1e6, 2), b.get('mirror')))"
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err; rc=$?
grep "^\[bench\]" $O/driver.err | tail -40 > $O/driver_progress.txt; echo "driver rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/driver.err; exit 1; }
python tools/sessions/r6/summarize.py $O
echo session done
