set -e
cd $GRAFT_REPO_ROOT
T=${1:-r03d}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_band_solve.py tests/test_gpu_loop_closure.py tests/test_gpu_configs.py > gpurun_out/$T.pytest.log 2>&1
timeout -k 10 300 python -u scripts/ab_compare.py --variant orig:AMC_LBA_LIB=amc-slam_amd/lib/exp/nodpp.so --variant pair: > gpurun_out/$T.ab1.log 2>&1
timeout -k 10 300 python -u scripts/ab_compare.py --config cfg2_global_500kf --calls 5 --variant orig:AMC_LBA_LIB=amc-slam_amd/lib/exp/nodpp.so --variant pair: > gpurun_out/$T.ab2.log 2>&1
timeout -k 10 200 python scripts/phase_times.py --out gpurun_out/${T}_phases.txt > gpurun_out/$T.ph.log 2>&1
