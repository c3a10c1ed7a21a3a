#!/bin/bash
# Build libbt_base.so from the library sources at git revision $1 (default HEAD), in a
# temporary worktree, for scripts/gpu_abl.sh.
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}; tmp=$(mktemp -d)
git worktree add -q --detach "$tmp" "$rev"
make -s -j8 -C "$tmp/distributed-backtesting-exploration_amd/csrc" OUT="$PWD/distributed-backtesting-exploration_amd/libbt_base.so" BUILD="$tmp/build"
git worktree remove --force "$tmp"
