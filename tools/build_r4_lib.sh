#!/bin/bash
# Build the round-4 product library (the RoIAlign forward with an 8-KB slab and per-lane
# global gathers for tap grids > 512 cells) as the A/B reference of tools/bench_roi_sets.py:
# tools/lib/r4/libfrcnn_amd_r4.so.  Runs here (hipcc cross-compiles gfx950); the .so travels
# to the GPU box with the tree.
set -euo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-792cef7}
WT=$(mktemp -d /tmp/frcnn_r4.XXXXXX)
git -C "$REPO" worktree add --detach "$WT" "$REV" >/dev/null
trap 'git -C "$REPO" worktree remove --force "$WT"; git -C "$REPO" worktree prune' EXIT
python "$WT/pytorch-faster-rcnn_amd/build_lib.py" >/dev/null
mkdir -p "$REPO/tools/lib/r4"
cp "$WT/pytorch-faster-rcnn_amd/frcnn_amd/libfrcnn_amd.so" "$REPO/tools/lib/r4/libfrcnn_amd_r4.so"
echo "$REPO/tools/lib/r4/libfrcnn_amd_r4.so"
