#!/bin/bash
# Build the LocalGPBA adapter (libamc_lba_map.so) from the sources of a git ref into amc-slam_amd/lib/exp/<name>.so,
# linked against the working tree's engine (A/B of adapter builds: AMC_LBA_MAP_LIB=amc-slam_amd/lib/exp/<name>.so,
# scripts/cmp_map_libs.py).
#   scripts/build_ref_map_lib.sh [ref=HEAD] [name=map_head]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REF=${1:-HEAD}
NAME=${2:-map_head}
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/amc-slam_amd/host" "$TMP/amc-slam_amd/csrc" "$TMP/include" "$ROOT/amc-slam_amd/lib/exp"
for f in $(git -C "$ROOT" ls-tree --name-only "$REF" amc-slam_amd/host/ amc-slam_amd/csrc/ include/); do
  git -C "$ROOT" show "$REF:$f" > "$TMP/$f"
done
H=$TMP/amc-slam_amd/host
g++ -O2 -std=c++17 -fPIC -shared -pthread -ffp-contract=off "$H/lba_map.cpp" "$H/optimizer.cpp" "$H/bundle_adjustment.cpp" \
    "$H/capi.cpp" -o "$ROOT/amc-slam_amd/lib/exp/$NAME.so" -L"$ROOT/amc-slam_amd/lib" -lamc_lba -Wl,-rpath,'$ORIGIN/..'
echo "built $ROOT/amc-slam_amd/lib/exp/$NAME.so from $REF"
