#!/bin/bash
# round-4 session check: the whole -m gpu suite (the fp32-residual tests print their deviations), an A/B of the
# t_s producers, and config 1 / 2 benches with and without the fp32-residual option
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
T=${1:-r4bd}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf --durations=20 --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
ROUNDS=2 STEPS=200 bash scripts/ab_envs.sh ${T}ab "" "LBA_NO_TS_PRE=1" "LBA_NO_LA_SPLIT=1" > gpurun_out/${T}_ab.txt 2>&1 || exit $?
for c in cfg1_local_50kf cfg2_global_500kf; do
  for f in "" "--f32-residual"; do
    timeout -k 10 400 python bench.py --config $c --steps 50 --warmup 5 --no-cpu $f > gpurun_out/${T}_${c}${f}.log 2>&1
    rc=$?; echo "bench $c $f rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
