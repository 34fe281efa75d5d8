#!/bin/bash
# PMC counters of the sweep kernel (default k_lin_schur) from rocprofv3, the way
# /opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE in separate passes
# (they do not fit one TCC pass), counters only (no other tracing), FETCH_SIZE doubled on gfx950; then
# one SQ pass (waves, busy cycles, VALU / LDS instructions, LDS bank conflicts).
# Writes gpurun_out/pmc_<tag>/ and gpurun_out/pmc_<kernel>_<tag>.json.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}
KERNEL=${KERNEL:-k_lin_schur}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run_pass() {   # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KERNEL" --output-format csv -d "$OUT/$name" -o pmc \
      -- python3 "$ROOT/bench.py" --config "${PMC_CONFIG:-cfg1_local_50kf}" --steps 10 --warmup 2 --no-cpu > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
run_pass FETCH_SIZE FETCH_SIZE || exit 1
run_pass WRITE_SIZE WRITE_SIZE || exit 1
run_pass SQ ${SQ_COUNTERS:-SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT} || exit 1
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" "$ROOT/gpurun_out/pmc_${KERNEL}_$TAG.json" "$KERNEL"
