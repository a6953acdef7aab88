# round 5, session 29: where a lone decode group's time goes -- empty-kernel lone time, the HBM
# group without CRC, one-window segments, at 1 / 4 / 8 parts
set -o pipefail
O=gpurun_out/r05_s29
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
for cfg in "16 128 200 1" "16 128 200 4" "16 128 200 8" "16 10 200 1" "64 10 200 1"; do
  n=$(echo $cfg | tr ' ' '_')
  timeout -k 10 120 tools/probes/bin/span_bench_v4 $cfg > $O/sb_$n.json 2> $O/sb_$n.err; rc=$?
  cat $O/sb_$n.json; echo; fatal $rc $n; [ $rc -eq 0 ] || { cat $O/sb_$n.err; exit 1; }
done
echo session done
