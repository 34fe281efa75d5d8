#!/bin/bash
# A/B of an environment switch on ONE GPU box: bench.py without / with `VAR=VALUE`, ROUNDS rounds.
#   gpurun -- 'bash scripts/ab_env.sh TAG LBA_NO_FUSED_EVAL=1'
set -u
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; KV=$2
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CFGS:-cfg1_local_50kf}; do
    for v in off on; do
      if [ $v = on ]; then E="env $KV"; else E=""; fi
      $E timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-200} --warmup 10 --no-cpu > gpurun_out/${T}_${c}_${v}_$r.bench.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
      python - gpurun_out/${T}_${c}_${v}_$r.bench.log "$v:$KV" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(f"{sys.argv[2]:28s} {d['config']['workload'].split(':')[0]:18s} value {d['value']:9.2f}  ms/step {d['ms_per_step']:.4f}  "
              f"sweep us {d['roofline']['avg_launch_ms'] * 1e3:8.2f}  solve us {d['roofline_solve']['avg_launch_ms'] * 1e3:8.2f}  "
              f"trials/step {d['trials_per_step']:.2f}", flush=True)
PY
    done
  done
done
