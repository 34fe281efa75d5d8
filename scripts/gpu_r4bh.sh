#!/bin/bash
# the whole -m gpu suite, then an A/B of the last-row solve shortcut (LBA_NO_LAST_ROW) on config 1 and config 2
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
T=${1:-r4bh}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --durations=10 --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 STEPS=200 bash scripts/ab_envs.sh ${T}ab "" "LBA_NO_LAST_ROW=1" > gpurun_out/${T}_ab.txt 2>&1 || exit $?
CFG=cfg2_global_500kf ROUNDS=1 STEPS=30 bash scripts/ab_envs.sh ${T}ab2 "" "LBA_NO_LAST_ROW=1" >> gpurun_out/${T}_ab.txt 2>&1 || exit $?
