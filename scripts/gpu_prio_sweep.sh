#!/bin/bash
# Wave-priority sweep of the EMA tile kernel (profiling library): BT_ABLATE bit 20 enables the
# override, bits 16-17 = the chain's priority, bits 18-19 = the walk's. CASES "symbols".
#   MASKS="0 1048576 ..." CASES="500 250" R=2 bash scripts/gpu_prio_sweep.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prio
for r in $(seq ${R:-2}); do
  for s in ${CASES:-500 250}; do
    for m in ${MASKS}; do
      BT_LIB=dev/prof.so BT_ABLATE=$m timeout -k 10 100 python3 bench.py --config ${CFG:-3} --symbols $s --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prio/b.log 2>&1 || { tail -5 gpurun_out/prio/b.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/prio/b.log').read().strip().splitlines()[-1]); m=$m; print('round $r symbols $s mask', m, 'chain', (m>>16)&3 if m>>20&1 else 3, 'walk', (m>>18)&3 if m>>20&1 else 2, 'kernel', round(d['roofline']['kernel_avg_ms'],4))"
    done
  done
done
