#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc2/counters_list.txt 2>&1
run() { local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc2/$name -o $name -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc2/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc; }
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
run sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH || exit 1
