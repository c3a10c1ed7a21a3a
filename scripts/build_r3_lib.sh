#!/bin/bash
# Builds the round-3 library (commit e255889, before the level-fill slack fix of round 4) as
# distributed-backtesting-exploration_amd/dev/r3.so, for the regression check in
# scripts/gpu_r05_a.sh (engine.py binds post-v2 symbols lazily, so it loads).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d)
BUILD=$(mktemp -d)
rmdir "$WT"
# the worktree is unregistered and the scratch build removed however the build ends
trap 'git -C "$ROOT" worktree remove --force "$WT" 2>/dev/null; rm -rf "$BUILD"' EXIT
git -C "$ROOT" worktree add -f "$WT" e255889 >/dev/null
make -s -j8 -C "$WT/distributed-backtesting-exploration_amd/csrc" \
    OUT="$ROOT/distributed-backtesting-exploration_amd/dev/r3.so" BUILD="$BUILD"
