#!/bin/bash
# LDS-layout A/B of k_lin_schur on one box: bitwise LM-run comparison, bench rounds, then one SQ counter pass
# (LDS instructions / bank conflicts / VALU / busy) per library.
#   gpurun -- 'bash scripts/gpu_r5_lds.sh TAG name...'   (name: lib/exp/<name>.so; "main" = the in-tree build)
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
T=$1; shift
X=$PWD/amc-slam_amd/lib/exp
for v in "$@"; do
  [ "$v" = main ] && continue
  timeout -k 10 300 python scripts/cmp_libs.py main $X/$v.so cfg1_local_50kf > gpurun_out/${T}_cmp_$v.txt 2>&1; rc=$?
  tail -2 gpurun_out/${T}_cmp_$v.txt; [ $rc -eq 0 ] || exit $rc
done
args=()
for v in "$@"; do if [ "$v" = main ]; then args+=(""); else args+=("AMC_LBA_LIB=$X/$v.so"); fi; done
ROUNDS=${ROUNDS:-2} STEPS=${STEPS:-200} bash scripts/ab_envs.sh ${T}ab "${args[@]}" > gpurun_out/${T}_ab.txt 2>&1; rc=$?
cat gpurun_out/${T}_ab.txt; [ $rc -eq 0 ] || exit $rc
[ -n "${SKIP_PMC:-}" ] && exit 0
for v in "$@"; do
  if [ "$v" = main ]; then unset AMC_LBA_LIB; else export AMC_LBA_LIB=$X/$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS \
      SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex k_lin_schur --output-format csv \
      -d $OLDPWD/gpurun_out/pmc_${T}_$v/SQ -o pmc -- python3 $OLDPWD/bench.py --steps 10 --warmup 2 --no-cpu \
      > $OLDPWD/gpurun_out/pmc_${T}_$v.log 2>&1); rc=$?
  echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/pmc_${T}_$v/SQ $v <<'PY'
import csv, glob, os, sys
vals = {}
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_lin_schur" in r.get("Kernel_Name", ""):
            vals.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
med = {c: sorted(d.values())[len(d) // 2] for c, d in vals.items()}
print(sys.argv[2], {c: round(v) for c, v in sorted(med.items())},
      "conflict/inst %.3f" % (med.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, med.get("SQ_INSTS_LDS", 1))))
PY
done
unset AMC_LBA_LIB
