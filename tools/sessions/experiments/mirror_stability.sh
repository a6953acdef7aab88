#!/bin/bash
# HBM-mirror stability: VarLen tokens (4 000 steps) with 1 and 2 copy streams, config 4 at both lengths
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ms
for rep in 1 2; do
  for n in 1 2; do
    TORCHKAFKA_MIRROR_COPY_STREAMS=$n timeout -k 10 200 python benchmarks/varlen_tokens.py --h2d dma > gpurun_out/ms/tok_s${n}_$rep.log 2>&1 || exit $?
    echo "tokens dma streams $n rep $rep: $(grep -o '"value": [0-9]*' gpurun_out/ms/tok_s${n}_$rep.log) $(grep -o '"mirror_fallbacks": [0-9]*' gpurun_out/ms/tok_s${n}_$rep.log)"
  done
  for st in 4000 20000; do
    timeout -k 10 200 python benchmarks/config4_json_varlen.py --steps $st > gpurun_out/ms/c4_${st}_$rep.log 2>&1 || exit $?
    echo "config4 $st rep $rep: $(grep -o '"value": [0-9]*' gpurun_out/ms/c4_${st}_$rep.log) $(grep -o '"mirror_fallbacks": [0-9]*' gpurun_out/ms/c4_${st}_$rep.log)"
  done
done
