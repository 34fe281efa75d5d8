#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py (config 1) with and without an environment switch, on ONE GPU box:
#   gpurun -- 'bash scripts/prof_env.sh TAG LBA_NO_FUSED_EVAL=1'
# writes gpurun_out/TAG_{base,env}/.../kernel_stats.csv and gpurun_out/TAG_{base,env}.txt (per-iteration view)
set -eu
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; KV=${2:-}
export TMPDIR=/tmp
for v in base env; do
  if [ $v = env ]; then [ -n "$KV" ] || break; export "$KV"; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_$v -o run -- python3 bench.py --steps ${STEPS:-100} \
      --warmup 10 --no-cpu ${BENCH_ARGS:-} > gpurun_out/${T}_$v.log 2>&1
  f=$(find gpurun_out/${T}_$v -name "*kernel_stats.csv" | head -1)
  python3 scripts/kstats.py "$f" $((${STEPS:-100} + 10 + 10)) > gpurun_out/${T}_$v.txt
done
