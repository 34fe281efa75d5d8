#!/bin/bash
# A/B of one environment setting on one GPU box with the working tree's library: bench.py alternately without
# and with "$ENV_B" (e.g. ENV_B="LBA_FLOW_FUSED=1"), twice.   gpurun -- 'ENV_B="X=1" bash scripts/env_ab.sh TAG'
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1
for v in a b a2 b2; do
  case $v in b*) E="$ENV_B";; *) E="";; esac
  env $E timeout -k 10 300 python bench.py --config ${CFG:-cfg1_local_50kf} --steps ${STEPS:-100} --warmup 10 --no-cpu > gpurun_out/${T}_$v.bench.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
  python - gpurun_out/${T}_$v.bench.log $v <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(f"{sys.argv[2]:3s} value {d['value']:9.2f}  ms/step {d['ms_per_step']:.4f}  sweep us {d['roofline']['avg_launch_ms'] * 1e3:7.2f}  "
              f"solve us {d['roofline_solve']['avg_launch_ms'] * 1e3:7.2f}  phases " + " ".join(f"{k} {x * 1e3:.1f}" for k, x in d['phases_ms_per_step'].items() if k != 'trials'))
PY
done
