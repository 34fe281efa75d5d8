#!/bin/bash
# A/B of lba_set_problem wall time on one GPU box: amc-slam_amd/lib/exp/head.so (scripts/build_ref_lib.sh) vs
# the working tree's library, alternately, 3 rounds (scripts/setup_phases_gpu.py, 6 set-ups each).
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
T=${1:-setup_ab}
for r in 1 2 3; do
  for v in head new; do
    case $v in head) export AMC_LBA_LIB=$PWD/amc-slam_amd/lib/exp/head.so;; *) unset AMC_LBA_LIB;; esac
    timeout -k 10 120 python scripts/setup_phases_gpu.py > gpurun_out/${T}_${v}_$r.log 2>&1 || exit 1
    echo "$v $r: $(grep wall gpurun_out/${T}_${v}_$r.log | awk '{print $3}' | tr '\n' ' ')"
  done
done
