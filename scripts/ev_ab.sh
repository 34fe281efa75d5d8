set -e
cd $GRAFT_REPO_ROOT
for m in every sampled off every sampled off; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu --sweep-events $m > gpurun_out/R3b_$m.log 2>&1
  python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/R3b_$m.log') if l.startswith('{')][0]; print('$m', round(d['value'],1), d['roofline']['avg_launch_ms'], d['roofline']['timed_launches'], d['roofline_solve']['avg_launch_ms'])"
done
