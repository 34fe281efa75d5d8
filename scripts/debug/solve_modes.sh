#!/bin/bash
# cfg1 / cfg2 bench with the L^-1 (dense) and substitution (band) solves side by side
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in cfg1_local_50kf cfg2_global_500kf; do
  for m in dense band; do
    timeout -k 10 300 python bench.py --config $cfg --solve $m --steps 20 --warmup 3 --no-cpu > gpurun_out/solve_${cfg}_${m}.log 2>&1 || exit $?
    echo "$cfg $m done"
  done
done
