#!/bin/bash
# Round 6 E8: EMA walk at the chain's priority (3), config 3 at 500 and 250 symbols.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/r; mkdir -p $O
export PYTHONUNBUFFERED=1
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 500 libbt.so dev/w3.so
ab 3 250 libbt.so dev/w3.so
