#!/bin/bash
# PMC passes over one config's per-GPU shard (bench.py --config): ./gpu_pmc_cfg.sh 4
cd "${GRAFT_REPO_ROOT:-/root/repo}"; C=${1:-4}; O=gpurun_out/pmc_cfg$C; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o $name -- python3 bench.py --config $C --steps 2 --warmup 0 --no-cpu-baseline > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc; }
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
run sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH || exit 1
run grbm GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
python3 scripts/pmc_table.py $O
