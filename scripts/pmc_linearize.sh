#!/bin/bash
# HBM traffic of the sweep kernel (k_linearize) from rocprofv3 PMC counters, the way
# /opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE in separate
# passes (they do not fit one TCC pass), counters only (no other tracing), FETCH_SIZE doubled on
# gfx950.  Writes gpurun_out/pmc_<tag>/ and gpurun_out/pmc_k_linearize_<tag>.json.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex k_linearize --output-format csv -d "$OUT/$C" -o pmc \
      -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu > "$OUT/$C.log" 2>&1
  rc=$?
  echo "pmc $C rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" "$ROOT/gpurun_out/pmc_k_linearize_$TAG.json"
