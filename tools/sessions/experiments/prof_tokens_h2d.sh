cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/tokdma
for h in auto dma; do
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/tokdma/$h" -o run -- python3 "$OLDPWD/benchmarks/varlen_tokens.py" --h2d $h --steps 2000 > "$OLDPWD/gpurun_out/tokdma/$h.log" 2>&1) || exit $?
echo "== $h $(grep -o '"value": [0-9]*' gpurun_out/tokdma/$h.log)"
cut -d, -f1-4 gpurun_out/tokdma/$h/run_kernel_stats.csv | cut -c1-120 | head -3
head -3 gpurun_out/tokdma/$h/run_memory_copy_stats.csv | cut -d, -f1-4
grep -o '"mirror_mib_copied": [0-9.]*\|"mirror_fallbacks": [0-9]*\|"mirror_copies": [0-9]*' gpurun_out/tokdma/$h.log | tr '\n' ' '; echo
done
