"""One line per bench.py JSON result in a session directory: the steady blocks in M rec/s."""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    if "value" not in d:
        continue
    row = {"value": round(d["value"] / 1e6, 2)}
    for k in ("steady_state", "steady_dma", "steady_f32", "steady_label", "steady_shm", "steady_shm_sync",
              "steady_rccl", "steady_rccl_sync", "steady_verified", "steady_unverified"):
        if isinstance(d.get(k), dict):
            row[k] = round(d[k]["records_per_s"] / 1e6, 2)
            if "batches_per_commit" in d[k]:
                row[k + "_bpc"] = d[k]["batches_per_commit"]
            if "lockstep_wait_us_per_step" in d[k]:
                row[k + "_wait_us"] = d[k]["lockstep_wait_us_per_step"]
    b = d.get("bridge") or {}
    for k in ("async", "sync", "lz4", "zstd"):
        if isinstance(b.get(k), dict):
            row["bridge_" + k] = round(b[k]["records_per_s"] / 1e6, 2)
    print(f.split("/")[-1], json.dumps(row))
