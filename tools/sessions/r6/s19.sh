# round 6, session 19: where the compressed bridge blocks' CPU goes (VERDICT r5 "do this" 7: lz4 / zstd
# at 10-15 M against the probe's 17-21 M) -- a per-thread-name census (TK_BENCH_CPU=1) of the lz4 and
# zstd blocks, twice, beside the uncompressed async block of the same process
set -o pipefail
O=gpurun_out/r06_s19
mkdir -p $O
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null || true
for rep in 1 2; do
  n=codecs_$rep
  TK_BENCH_CPU=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks "" --config-blocks "" --bridge-codecs lz4,zstd > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
done
python - <<'PY' | tee gpurun_out/r06_s19/census.txt
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_s19/codecs_*.json")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    br = j.get("bridge") or {}
    for k, b in br.items():
        if not (isinstance(b, dict) and "records_per_s" in b):
            continue
        c = b.get("cpu", {})
        print(f.split("/")[-1], k, round(b["records_per_s"] / 1e6, 2), "M rec/s; fill", b.get("worker_fill_us_per_batch"),
              "us/batch; cores", json.dumps(c.get("cores")))
        print("    by name:", json.dumps(c.get("by_name")))
        for key in ("wire_gb_per_s", "inflated_gb_per_s", "inflate_gb_per_s_per_thread", "fetch_thread_time_share",
                    "inflater_time_share", "producer", "fetch_threads", "inflate_threads"):
            if key in b:
                print("    ", key, json.dumps(b[key]))
PY
echo session done
