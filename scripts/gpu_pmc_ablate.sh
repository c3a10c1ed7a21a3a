#!/bin/bash
# SQ counters of the config-2 SMA kernel with phases removed (BT_ABLATE masks; outputs wrong by
# design): where the VALU / LDS instructions and LDS cycles go. One counter group per run.
export BT_LIB=${BT_LIB:-dev/prof.so}  # profiling build (make PROFILING=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmca
export TMPDIR=/tmp
for m in ${MASKS:-0 1 2 4 8 12 15}; do
  for g in 1 2; do
    if [ $g = 1 ]; then C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"
    else C="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; fi
    BT_ABLATE=$m timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmca/m${m}g$g -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmca/m${m}g$g.log 2>&1
    rc=$?; echo "mask $m group $g rc=$rc"; [ $rc = 0 ] || exit $rc
  done
done
