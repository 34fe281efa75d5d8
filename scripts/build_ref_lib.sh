#!/bin/bash
# Build libamc_lba.so from the sources of a git ref into amc-slam_amd/lib/exp/<name>.so (A/B against the
# working tree on one GPU box: AMC_LBA_LIB=amc-slam_amd/lib/exp/<name>.so selects it).
#   scripts/build_ref_lib.sh [ref=HEAD] [name=head]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REF=${1:-HEAD}
NAME=${2:-head}
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$TMP/amc-slam_amd/csrc" "$TMP/include" "$ROOT/amc-slam_amd/lib/exp"
for f in $(git -C "$ROOT" ls-tree --name-only "$REF" amc-slam_amd/csrc/ include/); do
  git -C "$ROOT" show "$REF:$f" > "$TMP/$f"
done
C=$TMP/amc-slam_amd/csrc
EXTRA=""
[ -f "$C/lba_debug.hip" ] && EXTRA="$C/lba_debug.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$C/lba_kernels.hip" "$C/lba_host.hip" \
    "$C/lba_track.hip" $EXTRA -o "$ROOT/amc-slam_amd/lib/exp/$NAME.so" -lrccl
echo "built $ROOT/amc-slam_amd/lib/exp/$NAME.so from $REF"
