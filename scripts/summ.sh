#!/bin/bash
# summary of a gpu_check run: bench headline, kernel stats, phase table head
T=$1
python3 - "$T" <<'PY'
import json, csv, sys
t = sys.argv[1]
for l in open(f'gpurun_out/{t}.bench.log'):
    if l.startswith('{'):
        d = json.loads(l)
        print('value', round(d['value'], 1), 'ms/step', round(d['ms_per_step'], 4), 'sweep', d['roofline']['avg_launch_ms'],
              'frac', round(d['roofline']['frac'], 3), 'solve', d['roofline_solve']['avg_launch_ms'])
        print('phases', d.get('phases_ms_per_step'), d.get('localgpba_calls'))
try:
    for r in csv.DictReader(open(f'gpurun_out/prof_{t}/trace_kernel_stats.csv')):
        print(f"{r['Name'][:34]:36s} {r['Calls']:>5s} {float(r['AverageNs'])/1000:9.2f} us  {r['Percentage'][:5]}%")
except FileNotFoundError:
    pass
PY
[ -f gpurun_out/${T}_phases.txt ] && sed -n 1,25p gpurun_out/${T}_phases.txt
