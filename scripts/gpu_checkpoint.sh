cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/g1
bash scripts/gpu_tests.sh && \
timeout -k 10 300 python3 bench.py > gpurun_out/g1/bench.log 2>&1 && tail -1 gpurun_out/g1/bench.log && \
timeout -k 10 120 python3 scripts/stamps_tile.py 4 500 > gpurun_out/g1/stamps4.log 2>&1; cat gpurun_out/g1/stamps4.log
