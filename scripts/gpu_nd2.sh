#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
T=$1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_loop_closure.py tests/test_gpu_band_solve.py > gpurun_out/$T.pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|three laps|Error|assert" gpurun_out/$T.pytest.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/ab_nd.sh $T

