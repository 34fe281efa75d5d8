#!/bin/bash
# round 5: the whole -m gpu suite on the main build, then an A/B of the reduced solve on config 1 (and config 2):
# main build, LBA_NO_TOP_MASTER=1, and an experimental build (AMC_LBA_LIB=lib/exp/<EXP>.so, parity subset first)
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
T=${1:-r5ab}
EXP=${EXP:-spec}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --durations=10 --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -f amc-slam_amd/lib/exp/$EXP.so ]; then
  AMC_LBA_LIB=$PWD/amc-slam_amd/lib/exp/$EXP.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_parity.py tests/test_gpu_numerics_edges.py tests/test_gpu_fusion.py > gpurun_out/${T}_exp_pytest.log 2>&1
  rc=$?; echo "exp pytest rc=$rc"; tail -3 gpurun_out/${T}_exp_pytest.log; [ $rc -eq 0 ] || exit $rc
  ROUNDS=2 STEPS=200 bash scripts/ab_envs.sh ${T}ab "" "LBA_NO_TOP_MASTER=1" "AMC_LBA_LIB=$PWD/amc-slam_amd/lib/exp/$EXP.so" > gpurun_out/${T}_ab.txt 2>&1 || exit $?
else
  ROUNDS=2 STEPS=200 bash scripts/ab_envs.sh ${T}ab "" "LBA_NO_TOP_MASTER=1" > gpurun_out/${T}_ab.txt 2>&1 || exit $?
fi
cat gpurun_out/${T}_ab.txt
