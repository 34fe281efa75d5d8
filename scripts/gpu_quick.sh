#!/bin/bash
# Quick GPU iteration: a subset of the GPU tests, one bench line (no CPU baseline), the phase stamps.
#   gpurun -- 'bash scripts/gpu_quick.sh TAG'   (TESTS=... to choose the tests, PHASES=0 to skip stamps)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
T=$1
OUT=gpurun_out
mkdir -p $OUT
if [ "${TESTS:-x}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_track.py tests/test_extrinsic.py tests/test_heavy_landmarks.py} \
      > $OUT/$T.pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/$T.pytest.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu > $OUT/$T.bench.log 2>&1
rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
python - $OUT/$T.bench.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print('value', round(d['value'], 1), 'sweep us', round(d['roofline']['avg_launch_ms'] * 1e3, 2),
              'solve us', round(d['roofline_solve']['avg_launch_ms'] * 1e3, 2), 'phases', d.get('phases_ms_per_step'))
PY
if [ "${PHASES:-1}" = "1" ]; then
  timeout -k 10 300 python scripts/phase_times.py --out $OUT/${T}_phases.txt > $OUT/$T.phases.log 2>&1
  rc=$?; echo "phases rc=$rc"
  grep -A3 "k_update timeline" $OUT/${T}_phases.txt
fi
exit 0
