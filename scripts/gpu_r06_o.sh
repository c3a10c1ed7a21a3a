#!/bin/bash
# Round 6 E6: Bollinger accountant out of the task rounds. Bollinger GPU tests, then config 4
# A/Bs (round start / HEAD / HEAD with accountant tasks) at 500 and 250 symbols.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/o; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "boll or Boll or config4 or config34 or segment or narrow or edge or flood or trade" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 4 500 dev/base.so libbt.so dev/acct_tasks.so
ab 4 250 dev/base.so libbt.so dev/acct_tasks.so
