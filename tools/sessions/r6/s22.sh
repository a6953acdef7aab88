# round 6, session 22: stale cache lines after an SDMA rewrite (tools/probes/reread_stress.hip): a
# region read by every XCD, rewritten by a copy, then checked by a kernel with no stream dependency
# on the copy (variant 0, the mirror's no-wait policy), after a stream wait on the completed copy
# event (1), or behind a system-scope acquire fence in the kernel (2).  One process, then four.
set -o pipefail
O=gpurun_out/r06_s22
mkdir -p $O
B=tools/probes/bin/reread_stress
run() {
  local n=$1; shift
  timeout -k 10 120 $B "$@" > $O/$n.json 2> $O/$n.err; local rc=$?
  echo "$n rc=$rc $(cat $O/$n.json) $(head -c 300 $O/$n.err)"
  [ $rc -le 1 ] || exit 1
}
four() {
  local n=$1; shift
  local pids=()
  for k in 1 2 3 4; do timeout -k 10 180 $B "$@" > $O/${n}_$k.json 2> $O/${n}_$k.err & pids+=($!); done
  local worst=0
  for p in "${pids[@]}"; do wait $p; rc=$?; [ $rc -gt $worst ] && worst=$rc; done
  for k in 1 2 3 4; do echo "$n.$k $(cat $O/${n}_$k.json) $(head -c 300 $O/${n}_$k.err)"; done
  [ $worst -le 1 ] || { echo "$n worst rc=$worst"; exit 1; }
}
run v0_64k 5000 64 0
run v0_1m 2000 1024 0
run v1_64k 5000 64 1
run v2_64k 5000 64 2
four v0_x4 5000 64 0
echo session done
