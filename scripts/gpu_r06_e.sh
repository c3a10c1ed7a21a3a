#!/bin/bash
# Round 6: EMA stages templated (TS = 2 unsplit, 64-bar stages for bar segments). GPU suite, then
# interleaved A/Bs: config 3 at 250 symbols (split run) round start / HEAD (SEG TS 1) / SEG TS 2
# / SEG TS 1 with chain tasks; config 3 at 500 round start / HEAD; config 4 round start / HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/e; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 250 dev/base.so libbt.so dev/seg2.so dev/seg1ct.so
ab 3 500 dev/base.so libbt.so
ab 4 500 dev/base.so libbt.so
ab 4 250 dev/base.so libbt.so
