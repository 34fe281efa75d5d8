# A/B runs on one GPU box: the GPU tests of TESTS (default: parity, heavy landmarks, configs), then
# scripts/ab_compare.py with the given variants, then the phase profile
set -e
cd $GRAFT_REPO_ROOT
T=$1; shift
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py tests/test_heavy_landmarks.py tests/test_gpu_configs.py} > gpurun_out/$T.pytest.log 2>&1
timeout -k 10 300 python -u scripts/ab_compare.py "$@" > gpurun_out/$T.ab1.log 2>&1
if [ "${PHASES:-1}" = "1" ]; then timeout -k 10 200 python scripts/phase_times.py --out gpurun_out/${T}_phases.txt > gpurun_out/$T.ph.log 2>&1; fi
