#!/bin/bash
# Runs one gpurun call, re-submitting it only while the pool had no box for it (gpurun reports
# status=transient: nothing ran, nothing was charged).  A call that ran -- passed or failed -- is
# never repeated.  Usage: tools/gpurun_retry.sh <log> <timeout_s> '<command>'
log=$1; t=$2; cmd=$3
for attempt in 1 2 3 4 5 6 7 8 9 10; do
  timeout $((t + 900)) /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "^=== " "$log"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${wait_s:-240} + 20 ))
    continue
  fi
  echo "attempt $attempt rc=$rc" >> "$log"
  exit $rc
done
echo "gave up: no box after 10 attempts" >> "$log"
exit 3
