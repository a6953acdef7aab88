# round 6, session 4: (1) the Kafka-protocol bridge alone on the box's CPUs (tools/probes/bridge_probe.py:
# where compressed topics are bound), (2) the RCCL lockstep blocks with the agreement captured into a
# HIP graph per slot against the three launches, (3) a kernel trace of config 4 (the JSON kernels)
set -o pipefail
O=gpurun_out/r06_s4
mkdir -p $O
timeout -k 10 300 python tools/probes/bridge_probe.py --records 300000 > $O/bridge_probe.log 2>&1; rc=$?
tail -4 $O/bridge_probe.log | cut -c1-400; echo "bridge probe rc=$rc"; [ $rc -eq 0 ] || exit 1
for mode in kernel graph; do
  TORCHKAFKA_RCCL_WORDS=$mode timeout -k 10 240 python bench.py --steps 20 --warmup 5 --steady-steps 2000 --extra-steps 20000 --extra-blocks rccl_sync,rccl,shm_sync --config-blocks "" --bridge-steps 0 > $O/rccl_$mode.json 2> $O/rccl_$mode.err; rc=$?
  echo "rccl $mode rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/rccl_$mode.err; exit 1; }
done
python - $O <<'PY'
import json, sys
for m in ("kernel", "graph"):
    d = json.loads(open(f"{sys.argv[1]}/rccl_{m}.json").read().strip().splitlines()[-1])
    for k in ("steady_rccl_sync", "steady_rccl", "steady_shm_sync"):
        b = d[k]
        print(m, k, round(b["records_per_s"] / 1e6, 2), "M", "wait/step", b.get("lockstep_wait_us_per_step"),
              "issue/step", b.get("lockstep_issue_us_per_step"), "bpc", b.get("batches_per_commit"),
              "words", b.get("lockstep", {}).get("words"))
PY
# the RCCL lockstep with 2 decode streams (one sharing a queue) against the fitted 1; coalesce 8 vs 6
TORCHKAFKA_RCCL_WORDS=graph timeout -k 10 240 python bench.py --steps 20 --warmup 5 --steady-steps 2000 --extra-steps 20000 --extra-blocks rccl --decode-streams 2 --config-blocks "" --bridge-steps 0 > $O/rccl_graph_ds2.json 2> $O/rccl_graph_ds2.err || exit 1
for c in 6 8; do
  for rep in 1 2; do
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --extra-blocks f32,label --coalesce $c --config-blocks "" --bridge-steps 0 > $O/coal${c}_$rep.json 2> $O/coal${c}_$rep.err || exit 1
  done
done
python tools/sessions/r6/summarize.py $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python benchmarks/config4_json_varlen.py --steps 4000 > $O/prof_c4.json 2> $O/prof_c4.err; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_c4.err; exit 1; }
db=$(ls $O/prof/*/*.db $O/prof/*.db 2>/dev/null | head -1)
python tools/rocpd_summary.py $db --md $O/kernels_c4.md > /dev/null && head -12 $O/kernels_c4.md
rm -f $db
echo session done
