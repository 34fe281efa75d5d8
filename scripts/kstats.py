"""Print a rocprofv3 kernel_stats.csv summary (per-iteration view)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iters = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    t = float(r["TotalDurationNs"])
    print(f"{r['Name'][:58]:58s} calls={int(r['Calls']):6d} avg_us={float(r['AverageNs'])/1e3:8.2f} "
          f"per_iter_us={t/1e3/iters:8.2f} pct={100*t/tot:6.2f}")
print(f"total per iter us = {tot/1e3/iters:.1f}")
