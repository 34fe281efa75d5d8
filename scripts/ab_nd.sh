#!/bin/bash
# A/B of two library builds on the bench's configs 2 and 4 (same box)
set -u
cd $GRAFT_REPO_ROOT
T=$1
for c in cfg2_global_500kf ${CFG4:-}; do
  for v in head new head2 new2; do
    case $v in head*) export AMC_LBA_LIB=$GRAFT_REPO_ROOT/amc-slam_amd/lib/exp/head.so;; *) unset AMC_LBA_LIB;; esac
    timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu > gpurun_out/${T}_${c}_$v.bench.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
    python - gpurun_out/${T}_${c}_$v.bench.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[2], d['config']['workload'].split(':')[0], 'value', round(d['value'], 2), 'ms/step', round(d['ms_per_step'], 3),
              'sweep ms', round(d['roofline']['avg_launch_ms'], 3), 'solve ms', round(d['roofline_solve']['avg_launch_ms'], 3),
              'trials/step', d['trials_per_step'], 'phases', d.get('phases_ms_per_step'))
PY
  done
done
