#!/bin/bash
# A/B of the working tree's library against amc-slam_amd/lib/exp/head.so (scripts/build_ref_lib.sh) on one
# GPU box: bench.py alternately head / new, twice, on each config of CFGS (default cfg1_local_50kf).
#   gpurun -- 'bash scripts/ab_bench.sh TAG'
set -u
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1
for c in ${CFGS:-cfg1_local_50kf}; do
  for v in head new head2 new2; do
    case $v in head*) export AMC_LBA_LIB=$PWD/amc-slam_amd/lib/exp/head.so;; *) unset AMC_LBA_LIB;; esac
    timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-200} --warmup 10 --no-cpu > gpurun_out/${T}_${c}_$v.bench.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
    python - gpurun_out/${T}_${c}_$v.bench.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(f"{sys.argv[2]:6s} {d['config']['workload'].split(':')[0]:18s} value {d['value']:9.2f}  ms/step {d['ms_per_step']:.4f}  "
              f"sweep us {d['roofline']['avg_launch_ms'] * 1e3:8.2f}  solve us {d['roofline_solve']['avg_launch_ms'] * 1e3:8.2f}  "
              f"trials/step {d['trials_per_step']:.2f}")
PY
  done
done
