#!/bin/bash
# E11 (64-bit DPP scans as add-with-carry pairs, dev/e11.so) against HEAD (libbt.so): the whole
# -m gpu suite on dev/e11.so, interleaved A/Bs on configs 2-4, the config-4 skeleton ablation.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06/x; mkdir -p $O
BT_LIB=dev/e11.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/e11_pytest_gpu.log 2>&1
rc=$?; tail -3 $O/e11_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for spec in "4 500" "3 500" "3 250" "4 250" "2 5000"; do
  set -- $spec
  ROUNDS=5 STEPS=5 timeout -k 10 300 python3 scripts/ab_inproc.py $1 $2 libbt.so dev/e11.so > $O/ab$1_$2.txt 2>&1
  rc=$?; grep config $O/ab$1_$2.txt; [ $rc -eq 0 ] || exit $rc
done
for lib in prof.so prof_e11.so; do
  BT_LIB=dev/$lib BT_ABLATE=10 timeout -k 10 200 python3 bench.py --config 4 --symbols 500 --steps 10 --warmup 2 --no-cpu-baseline --topk 0 > $O/skel_$lib.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/skel_$lib.log').read().strip().splitlines()[-1]); print('skeleton $lib kernel', round(d['roofline']['kernel_avg_ms'],4))"
done
