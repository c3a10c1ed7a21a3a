#!/bin/bash
# Builds the release library of a past commit as distributed-backtesting-exploration_amd/dev/NAME.so
# (an A/B arm for scripts/ab_inproc.py).   usage: scripts/build_ref_lib.sh COMMIT NAME
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
COMMIT=$1; NAME=$2
WT=$(mktemp -d); BUILD=$(mktemp -d); rmdir "$WT"
trap 'git -C "$ROOT" worktree remove --force "$WT" 2>/dev/null; rm -rf "$BUILD"' EXIT
git -C "$ROOT" worktree add -f "$WT" "$COMMIT" >/dev/null
mkdir -p "$ROOT/distributed-backtesting-exploration_amd/dev"
make -s -j8 -C "$WT/distributed-backtesting-exploration_amd/csrc" \
    OUT="$ROOT/distributed-backtesting-exploration_amd/dev/$NAME.so" BUILD="$BUILD"
