#!/bin/bash
# One GPU session: smoke -> gpu parity tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash (not a plain test failure) ends the script.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
TAG=${1:-run}
STEPS=${STEPS:-20}
echo "== smoke" | tee "$OUT/$TAG.status"
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/$TAG.smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/$TAG.status"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -rf --durations=40 --timeout 600 --timeout-method thread > "$OUT/$TAG.pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/$TAG.status"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 > "$OUT/$TAG.bench.log" 2>&1
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/$TAG.status"
[ $rc -eq 0 ] || exit $rc
if [ "${PHASES:-0}" = "1" ]; then
  timeout -k 10 300 python scripts/phase_times.py --out "$OUT/${TAG}_phases.txt" > "$OUT/$TAG.phases.log" 2>&1
  rc=$?; echo "phases rc=$rc" | tee -a "$OUT/$TAG.status"
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o trace \
      -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu > "$OUT/$TAG.prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/$TAG.status"
fi
exit 0
