#!/bin/bash
# rocprofv3 kernel-trace summaries + PMC (FETCH/WRITE/SQ) of the config 3/4/5 per-GPU shards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/prof_cfgs; mkdir -p $O
export TMPDIR=/tmp
for c in ${CFGS:-3 4 5}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace$c -o trace -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/trace$c.log 2>&1 || { echo "trace $c failed"; tail -5 $O/trace$c.log; exit 1; }
  echo "trace $c ok"
  for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $O/pmc$c/$n -o $n -- python3 bench.py --config $c --steps 2 --warmup 0 --no-cpu-baseline > $O/pmc${c}_$n.log 2>&1 || { echo "pmc $c $n failed"; exit 1; }
  done
  echo "pmc $c ok"
done
