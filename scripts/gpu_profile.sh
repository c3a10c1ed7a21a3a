#!/bin/bash
# Round profile: GPU tests, smoke, bench (with CPU baseline), rocprofv3 kernel-trace/stats,
# and PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) on the same bench command. Outputs in gpurun_out/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ge 2 ]; then echo "stopping after $name"; exit $rc; fi; return 0; }
step pytest_gpu 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python -u bench.py
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d gpurun_out/prof/sq -o sq -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_grbm 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/prof/grbm -o grbm -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
echo done
