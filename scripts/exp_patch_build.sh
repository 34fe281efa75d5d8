#!/bin/bash
# Build an experimental library from a patched COPY of the sources (the tree's sources, and so the main build's
# content stamp, stay untouched): scripts/exp_patch_build.sh NAME PATCH.py [-DFLAG...]
#   PATCH.py edits the copy in place: it receives the copy's csrc directory as argv[1].
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; PATCH=$2; shift 2
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/amc-slam_amd" "$ROOT/amc-slam_amd/lib/exp"
cp -r "$ROOT/amc-slam_amd/csrc" "$TMP/amc-slam_amd/csrc"
cp -r "$ROOT/include" "$TMP/include"
python3 "$PATCH" "$TMP/amc-slam_amd/csrc"
C=$TMP/amc-slam_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" "$C/lba_kernels.hip" "$C/lba_host.hip" \
    "$C/lba_track.hip" "$C/lba_debug.hip" -o "$ROOT/amc-slam_amd/lib/exp/$NAME.so" -lrccl
echo "built $ROOT/amc-slam_amd/lib/exp/$NAME.so"
