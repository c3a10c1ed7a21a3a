#!/bin/bash
# Round 6: config 3 split run (250 symbols): round start / HEAD / HEAD with the round-start ring
# size (dev/ring.so, valid for 64-bar stages only) / HEAD with chain tasks.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/i; mkdir -p $O
export PYTHONUNBUFFERED=1
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 250 dev/base.so libbt.so dev/ring.so dev/seg1ct.so
