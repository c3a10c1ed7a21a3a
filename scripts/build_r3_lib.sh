#!/bin/bash
# Builds the round-3 library (commit e255889, before the level-fill slack fix of round 4) as
# distributed-backtesting-exploration_amd/libbt_r3.so, for the regression check in
# scripts/gpu_r05_a.sh (engine.py binds post-v2 symbols lazily, so it loads).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/r3wt /tmp/r3build
git -C "$ROOT" worktree add -f /tmp/r3wt e255889 >/dev/null
make -s -j8 -C /tmp/r3wt/distributed-backtesting-exploration_amd/csrc \
    OUT="$ROOT/distributed-backtesting-exploration_amd/libbt_r3.so" BUILD=/tmp/r3build
git -C "$ROOT" worktree remove --force /tmp/r3wt
