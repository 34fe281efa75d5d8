#!/bin/bash
# A/B of engine builds on the GPU box: bitwise LM comparison of every variant against the first (scripts/cmp_libs.py),
# then interleaved bench.py rounds.  Variants are amc-slam_amd/lib/exp/<name>.so (scripts/exp_build.sh).
#   TAG=r8o VARIANTS="head la16" CONFIGS="cfg1_local_50kf cfg2_global_500kf" ROUNDS=2 S=100 bash scripts/ab_libs.sh
# Output: gpurun_out/<TAG>_ab.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
E=$PWD/amc-slam_amd/lib/exp
OUT=gpurun_out/${TAG}_ab.txt
mkdir -p gpurun_out
set -- $VARIANTS
BASE=$1; shift
: > "$OUT"
for c in ${CMP_CONFIGS:-$CONFIGS}; do
  for v in "$@"; do
    timeout -k 10 300 python scripts/cmp_libs.py "$E/$v.so" "$E/$BASE.so" "$c" >> "$OUT" 2>&1 || exit 1
  done
done
for c in $CONFIGS; do
  case $c in cfg1*) W=5;; cfg0*) W=5;; *) W=2;; esac
  case $c in cfg4*) ST=10;; cfg2*) ST=${S2:-20};; *) ST=${S:-100};; esac
  for r in $(seq 1 "${ROUNDS:-2}"); do
    for v in $VARIANTS; do
      echo -n "$c $v: " >> "$OUT"
      AMC_LBA_LIB=$E/$v.so timeout -k 10 300 python bench.py --config "$c" --steps "$ST" --warmup "$W" --no-cpu 2>/dev/null \
        | grep "^{" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],2), 'ms/step', round(d['ms_per_step']*1e3,2), 'solve us', round(d['roofline_solve']['avg_launch_ms']*1e3,1), 'sweep us', round(d['roofline_sweep']['avg_launch_ms']*1e3,1), 'trials', d['trials_per_step'])" >> "$OUT" || exit 1
    done
  done
done
echo "ab done" >> "$OUT"
