#!/bin/bash
# E11b (the DPP add-with-carry scans as non-volatile asm, dev/e11b.so) against HEAD (libbt.so)
# and E11 (dev/e11.so): the -m gpu suite on e11b, then three-arm interleaved A/Bs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06/y; mkdir -p $O
BT_LIB=dev/e11b.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/e11b_pytest_gpu.log 2>&1
rc=$?; tail -2 $O/e11b_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for spec in "4 500" "3 500" "2 5000" "3 250" "4 250"; do
  set -- $spec
  ROUNDS=6 STEPS=5 timeout -k 10 300 python3 scripts/ab_inproc.py $1 $2 libbt.so dev/e11.so dev/e11b.so > $O/ab$1_$2.txt 2>&1
  rc=$?; grep config $O/ab$1_$2.txt; [ $rc -eq 0 ] || exit $rc
done
