#!/bin/bash
# Round 6: split-run EMA kernel with records addressed on demand (fewer live VGPRs). GPU tests of
# EMA / segments, then config 3 A/Bs at 250 (split) and 500 symbols.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/l; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_segments.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shards.py -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 250 dev/base.so dev/basecho.so libbt.so dev/seg2.so
ab 3 500 dev/base.so libbt.so
