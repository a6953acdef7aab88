# round 6, session 10: where the CPU goes while the RCCL lockstep runs async at world 1 (its
# workers fill a batch in 25-39 us against 10-12 us in the same process's steady block, s8/s9):
# per-thread CPU of the main process and the workers over each block (TK_BENCH_CPU=1)
set -o pipefail
O=gpurun_out/r06_s10
mkdir -p $O
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/nproc.txt
for rep in 1 2; do
  TK_BENCH_CPU=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-steps 50000 --extra-blocks rccl,shm --config-blocks "" --bridge-steps 0 > $O/cpu_$rep.json 2> $O/cpu_$rep.err; rc=$?
  echo "cpu_$rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/cpu_$rep.err; exit 1; }
done
python - <<'PY'
import json
for r in (1, 2):
    j = json.loads(open(f"gpurun_out/r06_s10/cpu_{r}.json").read().strip().splitlines()[-1])
    for k in ("steady_state", "steady_rccl", "steady_shm"):
        b = j[k]
        print(r, k, round(b["records_per_s"] / 1e6, 2), "fill", b["worker_fill_us_per_batch"], json.dumps(b.get("cpu", {}).get("cores")),
              b.get("cpu", {}).get("affinity"))
        for t in b.get("cpu", {}).get("threads", [])[:8]:
            print("    ", t)
PY
echo session done
