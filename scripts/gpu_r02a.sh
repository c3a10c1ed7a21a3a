cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02a/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r02a/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02a/bench.log 2>&1 || exit 1
cat gpurun_out/r02a/bench.log
