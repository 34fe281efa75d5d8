#!/bin/bash
# Build an experimental variant of libamc_lba.so with extra defines into amc-slam_amd/lib/exp/<name>.so
# (load it with AMC_LBA_LIB=<path>): e.g. scripts/exp_build.sh nostore -DLBA_EXP_NOSTORE
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$ROOT/amc-slam_amd/lib/exp"
C=$ROOT/amc-slam_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" "$C/lba_kernels.hip" "$C/lba_host.hip" \
    "$C/lba_track.hip" "$C/lba_debug.hip" -o "$ROOT/amc-slam_amd/lib/exp/$NAME.so" -lrccl
