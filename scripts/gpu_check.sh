#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout (rc >= 2) ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu ${T_PYTEST:-500} python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_ARGS:-}
step smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python -u bench.py --steps 10 --warmup 2
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
find gpurun_out/prof -name "*stats*" | head
