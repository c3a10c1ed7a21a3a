#!/bin/bash
# Round 6: whole GPU suite at HEAD (EMA stages by the LDS rule for split and unsplit runs, A/B
# switches deleted), then interleaved A/Bs of configs 3 and 4 vs the round start.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/n; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 500 dev/base.so libbt.so
ab 3 250 dev/base.so libbt.so
