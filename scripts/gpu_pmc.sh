#!/bin/bash
# PMC passes over the config-2 bench (one counter group per rocprofv3 run; no trace domains).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() {  # run NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o $name -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
run sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run grbm GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
ls -R gpurun_out/pmc | head -40
