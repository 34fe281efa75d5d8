#!/bin/bash
# A/B/... of several library builds on ONE GPU box: bench.py with each amc-slam_amd/lib/exp/<name>.so in turn
# (names as arguments after the tag; "tree" = the working tree's library), ROUNDS rounds, on each config of CFGS.
#   gpurun -- 'bash scripts/ab_multi.sh TAG mode0 mode1 tree'
set -u
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; shift
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CFGS:-cfg1_local_50kf}; do
    for v in "$@"; do
      if [ "$v" = tree ]; then unset AMC_LBA_LIB; else export AMC_LBA_LIB=$PWD/amc-slam_amd/lib/exp/$v.so; fi
      timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-200} --warmup 10 --no-cpu > gpurun_out/${T}_${c}_${v}_$r.bench.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
      python - gpurun_out/${T}_${c}_${v}_$r.bench.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(f"{sys.argv[2]:8s} {d['config']['workload'].split(':')[0]:18s} value {d['value']:9.2f}  ms/step {d['ms_per_step']:.4f}  "
              f"sweep us {d['roofline']['avg_launch_ms'] * 1e3:8.2f}  solve us {d['roofline_solve']['avg_launch_ms'] * 1e3:8.2f}  "
              f"trials/step {d['trials_per_step']:.2f}", flush=True)
PY
    done
  done
done
