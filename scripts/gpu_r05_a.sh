#!/bin/bash
# Round 5, first GPU call: (1) the deep-wick narrow-accounts test against the round-3 library
# (libbt_r3.so, built from commit e255889 by scripts/build_r3_lib.sh), which must fail on a
# field mismatch of a wick series (the int32 accountant overflow of ADVICE r3), not on a
# missing symbol; (2) the whole -m gpu suite at HEAD; (3) the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
BT_LIB=libbt_r3.so timeout -k 10 300 $T tests/test_gpu_narrow.py -m gpu -k level_fills > gpurun_out/r05/narrow_r3lib.log 2>&1
rc=$?
echo "round-3 library: rc=$rc"
if [ $rc -ne 1 ]; then tail -20 gpurun_out/r05/narrow_r3lib.log; exit 3; fi
if grep -q "AttributeError\|undefined symbol" gpurun_out/r05/narrow_r3lib.log; then echo "failed for a wrong reason"; exit 4; fi
grep -E "^E +AssertionError: wick series [0-9]+ .*(mdd|pnl|n_trades|exposure|hash|sharpe)" gpurun_out/r05/narrow_r3lib.log | head -3 || { echo "no field mismatch in the log"; exit 5; }
timeout -k 10 900 $T tests -m gpu > gpurun_out/r05/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r05/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r05/pytest_gpu.log
timeout -k 10 300 python3 bench.py > gpurun_out/r05/bench_default.log 2>&1 || { tail -20 gpurun_out/r05/bench_default.log; exit 1; }
tail -1 gpurun_out/r05/bench_default.log | cut -c1-600
