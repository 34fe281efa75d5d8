#!/bin/bash
# rocprofv3 kernel-trace stats of the main build and of lib/exp/<name>.so builds, same command each (25 steps)
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
T=$1; shift
for v in main "$@"; do
  if [ "$v" = main ]; then E=""; else E="AMC_LBA_LIB=$PWD/amc-slam_amd/lib/exp/$v.so"; fi
  (cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/gpurun_out/prof_${T}_$v -o run -- python3 $OLDPWD/bench.py --steps 25 --warmup 3 --no-cpu > $OLDPWD/gpurun_out/${T}_${v}_prof.log 2>&1) || exit $?
  f=$(ls gpurun_out/prof_${T}_$v/run_kernel_stats.csv gpurun_out/prof_${T}_$v/*/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "== $v"; python scripts/kstats.py $f 48 | head -7 | tee gpurun_out/${T}_${v}_kernel_stats.txt
done
