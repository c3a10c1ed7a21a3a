#!/bin/bash
# Round 6 E4: GPU suite at HEAD, interleaved A/B of config 3 (round start / E1 / E2 / HEAD = E4)
# at 500 and 250 symbols, stamps of config 3 at 500 and 250 symbols (split run: speculative pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/d; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for S in 500 250; do
  timeout -k 10 300 python3 scripts/ab_inproc.py 3 $S dev/base.so dev/e1.so dev/e2.so libbt.so > $O/ab3_$S.txt 2>&1 || { tail -5 $O/ab3_$S.txt; exit 1; }
  grep -v amdgpu.ids $O/ab3_$S.txt
done
for S in 500 250; do
  timeout -k 10 200 python3 scripts/stamps_tile.py 3 $S > $O/stamps3_$S.txt 2>&1 || { tail -5 $O/stamps3_$S.txt; exit 1; }
  grep -v amdgpu.ids $O/stamps3_$S.txt
done
