#!/bin/bash
# Round 6 E2/E3: the EMA and Bollinger GPU tests at HEAD, then interleaved in-process A/Bs
# (scripts/ab_inproc.py): round start (dev/base.so) vs E1 (dev/e1.so) vs HEAD on config 3,
# round start vs HEAD on config 4; stamps of config 3 at HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/c; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 scripts/ab_inproc.py 3 500 dev/base.so dev/e1.so libbt.so > $O/ab3_500.txt 2>&1 || { tail -5 $O/ab3_500.txt; exit 1; }
cat $O/ab3_500.txt
timeout -k 10 300 python3 scripts/ab_inproc.py 3 250 dev/base.so dev/e1.so libbt.so > $O/ab3_250.txt 2>&1 || { tail -5 $O/ab3_250.txt; exit 1; }
cat $O/ab3_250.txt
timeout -k 10 300 python3 scripts/ab_inproc.py 4 500 dev/base.so libbt.so > $O/ab4_500.txt 2>&1 || { tail -5 $O/ab4_500.txt; exit 1; }
cat $O/ab4_500.txt
timeout -k 10 200 python3 scripts/stamps_tile.py 3 > $O/stamps3.txt 2>&1 && cat $O/stamps3.txt
