#!/bin/bash
# A/B of experimental builds on one box: bitwise comparison of LM runs (scripts/cmp_libs.py) of lib/exp/$CMP_A vs
# $CMP_B, then bench.py rounds over "" (the main build) and each lib/exp/<name>.so given, then an optional test subset
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
T=$1; shift
X=$PWD/amc-slam_amd/lib/exp
if [ -n "${CMP:-}" ]; then
  set -- "$@"
  a=${CMP%,*}; b=${CMP#*,}
  la=$([ "$a" = main ] && echo main || echo $X/$a.so); lb=$([ "$b" = main ] && echo main || echo $X/$b.so)
  timeout -k 10 300 python scripts/cmp_libs.py $la $lb ${CMP_CFG:-cfg1_local_50kf} > gpurun_out/${T}_cmp.txt 2>&1; rc=$?
  cat gpurun_out/${T}_cmp.txt; [ $rc -eq 0 ] || exit $rc
fi
args=("")
for v in "$@"; do args+=("AMC_LBA_LIB=$X/$v.so"); done
ROUNDS=${ROUNDS:-2} STEPS=${STEPS:-200} bash scripts/ab_envs.sh ${T}ab "${args[@]}" > gpurun_out/${T}_ab.txt 2>&1; rc=$?
cat gpurun_out/${T}_ab.txt; [ $rc -eq 0 ] || exit $rc
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; exit $rc
fi
