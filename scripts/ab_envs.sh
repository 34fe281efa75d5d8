#!/bin/bash
# bench.py (config 1) under several environment settings on ONE GPU box, ROUNDS rounds:
#   gpurun -- 'bash scripts/ab_envs.sh TAG "" "LBA_X=1" "LBA_X=2"'   ("" = no setting)
set -u
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; shift
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for kv in "$@"; do
    i=$((i + 1))
    if [ -n "$kv" ]; then E="env $kv"; else E=""; fi
    $E timeout -k 10 300 python bench.py --config ${CFG:-cfg1_local_50kf} --steps ${STEPS:-200} --warmup 10 --no-cpu > gpurun_out/${T}_${i}_$r.bench.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$kv rc=$rc"; exit $rc; }
    python - gpurun_out/${T}_${i}_$r.bench.log "${kv:-base}" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(f"{sys.argv[2]:34s} value {d['value']:9.2f}  ms/step {d['ms_per_step']:.4f}  sweep us {d.get('roofline_sweep', d['roofline'])['avg_launch_ms'] * 1e3:8.2f}  "
              f"solve us {d['roofline_solve']['avg_launch_ms'] * 1e3:8.2f}  trials/step {d['trials_per_step']:.2f}", flush=True)
PY
  done
done
