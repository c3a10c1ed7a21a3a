#!/bin/bash
# Round 5, first GPU call: (1) the deep-wick narrow-accounts test against the round-3 library
# (dev/r3.so, built from commit e255889 by scripts/build_r3_lib.sh), which must fail on a
# field mismatch of a wick series (the int32 accountant overflow of ADVICE r3), not on a
# missing symbol; (2) the new trade-parallel Bollinger kernel's parity tests, then the whole
# -m gpu suite; (3) the default bench line; (4) config 4 phase ablation of the round-4 kernel
# (profiling build dev/prof_r4.so); (5) config 4 kernel times, round-4 kernel (dev/r4.so,
# commit 66f7b0c) vs HEAD, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
BT_LIB=dev/r3.so timeout -k 10 300 $T tests/test_gpu_narrow.py -m gpu -k level_fills > gpurun_out/r05/narrow_r3lib.log 2>&1
rc=$?
echo "round-3 library: rc=$rc"
if [ $rc -ne 1 ]; then tail -20 gpurun_out/r05/narrow_r3lib.log; exit 3; fi
if grep -q "AttributeError\|undefined symbol" gpurun_out/r05/narrow_r3lib.log; then echo "failed for a wrong reason"; exit 4; fi
grep -E "^E +AssertionError: wick series [0-9]+ .*(mdd|pnl|n_trades|exposure|hash|sharpe)" gpurun_out/r05/narrow_r3lib.log | head -3 || { echo "no field mismatch in the log"; exit 5; }
timeout -k 10 400 $T tests/test_gpu_parity.py -m gpu -k "boll or tile_strategies or lane_strategies or config34 or maximum" > gpurun_out/r05/boll_parity.log 2>&1 || { tail -40 gpurun_out/r05/boll_parity.log; exit 1; }
tail -2 gpurun_out/r05/boll_parity.log
timeout -k 10 900 $T tests -m gpu > gpurun_out/r05/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r05/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r05/pytest_gpu.log
timeout -k 10 300 python3 bench.py > gpurun_out/r05/bench_default.log 2>&1 || { tail -20 gpurun_out/r05/bench_default.log; exit 1; }
tail -1 gpurun_out/r05/bench_default.log | cut -c1-400
for ab in 0 8 2 10; do
  BT_LIB=dev/prof_r4.so BT_ABLATE=$ab timeout -k 10 200 python3 bench.py --config 4 --symbols 500 --steps 10 --warmup 2 --no-cpu-baseline --topk 0 > gpurun_out/r05/abl4_$ab.log 2>&1 || { tail -5 gpurun_out/r05/abl4_$ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/abl4_$ab.log').read().strip().splitlines()[-1]); print('r4 config 4 ablate', $ab, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
done
for lib in dev/r4.so libbt.so dev/r4.so libbt.so; do
  for s in 500 250; do
    BT_LIB=$lib timeout -k 10 200 python3 bench.py --config 4 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/c4_${lib}_$s.log 2>&1 || { tail -5 gpurun_out/r05/c4_${lib}_$s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r05/c4_${lib}_$s.log').read().strip().splitlines()[-1]); print('$lib config 4', $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3), 'ms/step', round(d['ms_per_step'],3))"
  done
done
