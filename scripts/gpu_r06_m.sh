#!/bin/bash
# Round 6: split-run EMA kernel storing the chain's start values at once. Segment / EMA tests,
# then config 3 at 250 (split): round start / HEAD (SEG 64-bar stages) / SEG 128-bar stages.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/m; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_segments.py tests/test_gpu_shards.py -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 250 dev/base.so libbt.so dev/seg2.so
