cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
(cd _bisect/old && TORCHKAFKA_NO_REBUILD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -k "h2d_modes" -v -p no:cacheprovider --timeout 120 --timeout-method thread > ../../gpurun_out/bisect_old.log 2>&1); echo "old rc=$?"
TORCHKAFKA_NO_REBUILD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -k "h2d_modes" -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bisect_new.log 2>&1; echo "new rc=$?"
grep -E "PASSED|FAILED" gpurun_out/bisect_old.log gpurun_out/bisect_new.log
