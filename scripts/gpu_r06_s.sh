#!/bin/bash
# Round 6 E9: EMA walk inputs of both tiles read per stage. EMA GPU tests, config 3 A/B at 500
# and 250 symbols (dev/e7.so = the previous commit).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/s; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "ema or EMA or config3 or config34 or segment or stage or narrow or edge" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 500 dev/e7.so libbt.so
ab 3 250 dev/e7.so libbt.so
timeout -k 10 200 python3 scripts/stamps_tile.py 3 500 > $O/stamps3_500.txt 2>&1 && grep -v amdgpu.ids $O/stamps3_500.txt
