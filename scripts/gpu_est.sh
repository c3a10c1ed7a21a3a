cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
BT_LIB=dev/est.so timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_segments.py -k ema "tests/test_gpu_shards.py::test_strong_scaling_shard_full_shape" -s > gpurun_out/est_tests.log 2>&1 || { tail -30 gpurun_out/est_tests.log; exit 1; }
grep -E "passed|failed|segments" gpurun_out/est_tests.log | tail -8
LIBS="libbt.so dev/est.so" CASES="3:250 3:500" R=3 timeout -k 10 400 bash scripts/gpu_ab.sh
