#!/bin/bash
# Round 6: LDS-free top-k histogram for small key counts. Top-k / parity GPU tests, then the bench
# lines (step vs kernel) of configs 3 (500, 250), 4 (500) and the driver's default (config 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/${OUT:-u}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
k() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); print('$n', 'kernel', round(d['roofline']['kernel_avg_ms'],4), 'step', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3))"
}
k c3_s500 --config 3 --symbols 500 --steps 20
k c3_s250 --config 3 --symbols 250 --steps 20
k c4_s500 --config 4 --symbols 500 --steps 20
k c2 --steps 20
k c3_s500b --config 3 --symbols 500 --steps 20
