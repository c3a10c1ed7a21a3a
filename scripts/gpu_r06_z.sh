#!/bin/bash
# E11 kept for the EMA helper's scan only (libbt.so) against HEAD before it (dev/head6.so): the
# -m gpu suite, then interleaved A/Bs on configs 2-4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06/z; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for spec in "3 500" "3 250" "4 500" "2 5000"; do
  set -- $spec
  ROUNDS=6 STEPS=5 timeout -k 10 300 python3 scripts/ab_inproc.py $1 $2 dev/head6.so libbt.so > $O/ab$1_$2.txt 2>&1
  rc=$?; grep config $O/ab$1_$2.txt; [ $rc -eq 0 ] || exit $rc
done
