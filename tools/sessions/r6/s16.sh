# round 6, session 16: a thread census (TK_BENCH_CPU=1) of the bridge's async block alone and after
# the other blocks (verdict r5 weak 3: 38-46 M after them against 50-51 M alone, worker fill up)
set -o pipefail
O=gpurun_out/r06_s16
mkdir -p $O
for rep in 1 2; do
  n=alone_$rep
  TK_BENCH_CPU=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --steady-steps 20000 --extra-blocks "" --config-blocks "" --bridge-codecs "" > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
  n=after_$rep
  TK_BENCH_CPU=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config-blocks "" --bridge-codecs "" > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.err; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_s16/*.json")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    blocks = {k: v for k, v in j.items() if isinstance(v, dict) and "records_per_s" in v}
    blocks.update({"bridge_" + k: v for k, v in (j.get("bridge") or {}).items() if isinstance(v, dict) and "records_per_s" in v})
    for k, b in blocks.items():
        c = b.get("cpu", {})
        print(f.split("/")[-1], k, round(b["records_per_s"] / 1e6, 2), "fill", b.get("worker_fill_us_per_batch"), json.dumps(c.get("cores")))
        if k.startswith("bridge"):
            print("    ", [(t["who"], t["name"], t["cores"]) for t in c.get("threads", [])[:12]])
PY
echo session done
