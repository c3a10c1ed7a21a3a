#!/bin/bash
# Round 6, first box: the GPU suite at HEAD (split_grp2 removed, four pipeline slots, two-deep
# N>1 bench), then the tile kernels' baselines on this box: release kernel times for configs 3
# and 4 (500 / 250 symbols), the per-tile stamps and the skeleton ablation (BT_ABLATE=10).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/a; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
k() {  # name, lib, ablate, bench args
  local n=$1 lib=$2 ab=$3; shift 3
  BT_LIB=$lib BT_ABLATE=$ab timeout -k 10 200 python3 bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); print('$n', 'kernel', round(d['roofline']['kernel_avg_ms'],4), 'step', round(d['ms_per_step'],4))"
}
k c4_s500 libbt.so 0 --config 4 --symbols 500
k c4_s250 libbt.so 0 --config 4 --symbols 250
k c3_s500 libbt.so 0 --config 3 --symbols 500
k c3_s250 libbt.so 0 --config 3 --symbols 250
k c4_s500_abl10 dev/prof.so 10 --config 4 --symbols 500 --topk 0
k c4_s500_abl0 dev/prof.so 0 --config 4 --symbols 500 --topk 0
timeout -k 10 200 python3 scripts/stamps_tile.py 4 > $O/stamps4.txt 2>&1 && cat $O/stamps4.txt
timeout -k 10 200 python3 scripts/stamps_tile.py 3 > $O/stamps3.txt 2>&1 && cat $O/stamps3.txt
