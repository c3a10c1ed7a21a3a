#!/bin/bash
# Round 6: config 3 split run (250): round start vs round start with helper B out of the task
# rounds (dev/basecho.so) vs HEAD; unsplit 500 the same three.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/k; mkdir -p $O
export PYTHONUNBUFFERED=1
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 250 dev/base.so dev/basecho.so libbt.so
ab 3 500 dev/base.so dev/basecho.so dev/ts1.so
