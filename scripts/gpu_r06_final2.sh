#!/bin/bash
# Round 6 end checks at the final HEAD: the full -m gpu suite, smoke() and the default bench line
# (the driver's own commands), logs under gpurun_out/final/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/bench_default.log 2>&1
rc=$?; tail -1 $O/bench_default.log | cut -c1-400; exit $rc
