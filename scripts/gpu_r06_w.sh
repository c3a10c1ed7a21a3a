#!/bin/bash
# E10 (pooled Bollinger accountant, dev/e10.so) against HEAD (libbt.so): interleaved A/B on the
# config-4 shards (summaries compared bit for bit), the Bollinger parity tests on dev/e10.so,
# then the 128-bar EMA stage tests and a deep random sweep on HEAD (scripts/gpu_r06_v.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06/w; mkdir -p $O
for S in 500 250; do
  ROUNDS=5 STEPS=5 timeout -k 10 300 python3 scripts/ab_inproc.py 4 $S libbt.so dev/e10.so > $O/ab4_$S.txt 2>&1
  rc=$?; cat $O/ab4_$S.txt | tail -3; [ $rc -eq 0 ] || exit $rc
done
BT_LIB=dev/prof_e10.so timeout -k 10 200 python3 scripts/stamps_tile.py 4 > $O/stamps4_e10.txt 2>&1
rc=$?; cat $O/stamps4_e10.txt; [ $rc -eq 0 ] || exit $rc
BT_LIB=dev/e10.so timeout -k 10 600 python3 -u -m pytest tests/test_tile_edge_trades.py tests/test_gpu_random.py tests/test_gpu_segments.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_narrow.py tests/test_gpu_trade_cap.py -m gpu -k "boll or config4 or split or narrow or cap" -x -q --timeout 300 --timeout-method thread > $O/e10_parity.log 2>&1
rc=$?; tail -3 $O/e10_parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r06_v.sh
