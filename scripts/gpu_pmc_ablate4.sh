#!/bin/bash
# SQ instruction counters of the config-4 Bollinger kernel (500 symbols) with phases removed
# (profiling build, BT_ABLATE masks: 8 no walks, 2 no flag tasks; outputs wrong by design).
export BT_LIB=${BT_LIB:-dev/prof.so}
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc4a
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
for m in ${MASKS:-0 8 2 10}; do
  BT_ABLATE=$m timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc4a/m$m -o p -- python3 bench.py --config 4 --symbols 500 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc4a/m$m.log 2>&1
  rc=$?; echo "mask $m rc=$rc"; [ $rc = 0 ] || exit $rc
done
