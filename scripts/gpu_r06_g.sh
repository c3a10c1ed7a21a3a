#!/bin/bash
# Round 6: where the split-run (bar segment) slowdown comes from. Config 3 A/Bs: 500 symbols
# round start / HEAD (TS 2) / HEAD forced to 64-bar stages; 250 symbols (split) round start / HEAD
# (SEG TS 1) / SEG TS 2 with table tasks / SEG TS 2 with tables on helper A.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/g; mkdir -p $O
export PYTHONUNBUFFERED=1
ab() { timeout -k 10 300 python3 scripts/ab_inproc.py "$@" > $O/ab_$1_$2.txt 2>&1 || { tail -5 $O/ab_$1_$2.txt; exit 1; }; grep -v amdgpu.ids $O/ab_$1_$2.txt; }
ab 3 500 dev/base.so libbt.so dev/ts1.so
ab 3 250 dev/base.so libbt.so dev/seg2.so dev/seg2nodt.so
