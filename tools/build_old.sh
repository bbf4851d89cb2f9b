#!/usr/bin/env bash
# Build librtrt.so of an earlier commit into build/old/ (for tools/ab.py --libs A/Bs):
#   tools/build_old.sh <commit> [dest-dir]
set -euo pipefail
C=${1:?commit}
DEST=${2:-build/old}
ROOT=$(git rev-parse --show-toplevel)
WT=$(mktemp -d /tmp/rtrt_old.XXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$C"
make -C "$WT" -s -j8 lib >/dev/null
mkdir -p "$ROOT/$DEST"
cp "$WT/real_time_ray_tracer_amd/librtrt.so" "$ROOT/$DEST/librtrt.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "$ROOT/$DEST/librtrt.so <- $C"
