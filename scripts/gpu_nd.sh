#!/bin/bash
# GPU tests of the solver layout + bench of configs 1, 2 and 4 (single GPU)
set -u
cd $GRAFT_REPO_ROOT
T=$1
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_band_solve.py tests/test_gpu_loop_closure.py tests/test_gpu_partition.py tests/test_gpu_configs.py} > gpurun_out/$T.pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$T.pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in cfg1_local_50kf cfg2_global_500kf ${CFG4:-}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu > gpurun_out/${T}_$c.bench.log 2>&1
  rc=$?; echo "bench $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python - gpurun_out/${T}_$c.bench.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(d['config']['workload'].split(':')[0], 'value', round(d['value'], 2), 'ms/step', round(d['ms_per_step'], 3),
              'sweep ms', round(d['roofline']['avg_launch_ms'], 3), 'solve ms', round(d['roofline_solve']['avg_launch_ms'], 3),
              'trials/step', d['trials_per_step'])
PY
done
