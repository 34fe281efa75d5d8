#!/bin/bash
# rocprofv3 kernel stats of bench.py for the in-tree library and experimental builds (amc-slam_amd/lib/exp/<name>.so):
#   bash scripts/prof_variants.sh TAG base nogp nolmk ...
# writes gpurun_out/pv_<TAG>_<variant>/ and prints per-kernel average durations of each variant
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  OUT=$ROOT/gpurun_out/pv_${TAG}_$v
  if [ "$v" = base ]; then LIBV=""; else LIBV=$ROOT/amc-slam_amd/lib/exp/$v.so; fi
  AMC_LBA_LIB=$LIBV timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o trace \
      -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu > "$OUT.log" 2>&1
  rc=$?
  echo "== $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/trace_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    print(f"   {r['Name'][:40]:42s} {int(r['Calls']):5d} {float(r['AverageNs'])/1000:9.2f} us")
PY
done
