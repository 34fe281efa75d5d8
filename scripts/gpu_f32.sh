set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32_residual.py tests/test_gpu_parity.py -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/r4bc_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in cfg1_local_50kf cfg2_global_500kf; do
  for f in "" "--f32-residual"; do
    timeout -k 10 400 python bench.py --config $c --steps 50 --warmup 5 --no-cpu $f > gpurun_out/r4bc_${c}${f}.log 2>&1
    rc=$?; echo "bench $c $f rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
