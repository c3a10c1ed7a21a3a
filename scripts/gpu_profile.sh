#!/bin/bash
# One profile of a bench.py command on the GPU box, all from the SAME command line:
#   1. rocprofv3 --kernel-trace --stats of `python3 bench.py ARGS` (its bench JSON line goes to
#      bench.log: kernel averages and ms_per_step come from one process);
#   2. separate --pmc passes (FETCH_SIZE; WRITE_SIZE; 8 SQ counters; 2 GRBM counters) of the same
#      command with fewer steps (MI355X_MICROARCH.md: one TCC size counter per pass).
# usage: bash scripts/gpu_profile.sh NAME [bench.py args...]   -> gpurun_out/prof/NAME/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
NAME=$1; shift
O=gpurun_out/prof/$NAME; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 bench.py "$@" > $O/bench.log 2>&1
rc=$?; if [ $rc -ne 0 ]; then echo "trace $NAME failed rc=$rc"; tail -5 $O/bench.log; exit $rc; fi
grep '^{' $O/bench.log | tail -1 | cut -c1-400
PM="--steps 3 --warmup 1 --no-cpu-baseline"
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $O/$n -o $n -- python3 bench.py "$@" $PM > $O/pmc_$n.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pmc $NAME $n failed rc=$rc"; tail -5 $O/pmc_$n.log; exit $rc; fi
done
echo "profile $NAME ok"
