"""lba_set_problem's host sub-phases (LBA_SETUP_TIMING stamps of lba_setup_host_profile: no device) per thread count,
min and median over repeats, config 1:  python scripts/setup_subprof.py [threads ...]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = """
import sys; sys.path.insert(0, %r)
import amc_lba
from amc_lba.synth import make_config_window
w = make_config_window('cfg1_local_50kf')
for _ in range(15): amc_lba.setup_host_profile(w)
""" % os.path.join(ROOT, "amc-slam_amd")
for th in (sys.argv[1:] or ["1", "8", "16"]):
    r = subprocess.run([sys.executable, "-c", CODE], env=dict(os.environ, LBA_SETUP_TIMING="1", LBA_SETUP_THREADS=th),
                       capture_output=True, text=True, timeout=300)
    d = collections.OrderedDict()
    for line in r.stderr.splitlines():
        m = re.match(r"\s*(set_problem )?(.*?)\s+([0-9.]+) ms", line)
        if m:
            d.setdefault((m.group(1) or "") + m.group(2).strip(), []).append(float(m.group(3)))
    print(f"== threads {th}")
    for k, v in d.items():
        v = sorted(v[3:]) or sorted(v)   # (the first set-ups warm the pool and the allocator)
        print(f"  {k:36s} min {v[0]:7.3f}  med {v[len(v) // 2]:7.3f} ms")
