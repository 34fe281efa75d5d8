"""A/B of lba_set_problem on the caller's windows: the LocalGPBA windows of keyframes 20..39 of a synthetic
40-keyframe, 4-camera map (normal and bLarge), set up one after another on one engine, 3 passes; median wall ms
and phases per library build (main = the in-tree library, or a path given as AMC_LBA_LIB).  GPU run.
    python scripts/setup_ab_map.py main amc-slam_amd/lib/exp/head.so"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAKE = r"""
import sys, pickle
sys.path.insert(0, %r)
from amc_lba import mapsnap as ms
snap = ms.make_map(n_kf=40, n_lm=8000, obs_per_lm=6, n_cam=4, seed=7)
m = ms.LocalGPBAMap(snap)
wins = {large: [m.build_window(kf, large=large)[0] for kf in range(20, 40)] for large in (False, True)}
pickle.dump(wins, open(sys.argv[1], "wb"))
""" % os.path.join(ROOT, "amc-slam_amd")
# (the windows are made by the adapter in a process of their own and read back from a file this script wrote, so
#  the timed processes load one engine library only)
CODE = r"""
import sys, time, json, pickle
import numpy as np
sys.path.insert(0, %r)
import amc_lba
wins_all = pickle.load(open(sys.argv[1], "rb"))
out = {}
for large in (False, True):
    wins = wins_all[large]
    p = amc_lba.Problem(wins[0])
    t, ph = [], []
    for rep in range(3):
        for W in wins:
            t0 = time.perf_counter(); p.set_window(W); t.append(time.perf_counter() - t0); ph.append(p.setup_phases())
    p.close()
    out["large" if large else "normal"] = {"ms": round(float(np.median(t)) * 1e3, 3),
        "phases": {k: round(float(np.median([d[k] for d in ph])), 3) for k in ph[0]}}
print(json.dumps(out))
""" % os.path.join(ROOT, "amc-slam_amd")
WIN_FILE = os.path.join(os.environ.get("TMPDIR", "/tmp"), "setup_ab_windows.pkl")
os.makedirs(os.path.dirname(WIN_FILE), exist_ok=True)
subprocess.run([sys.executable, "-c", MAKE, WIN_FILE], check=True, timeout=300)
for rnd in range(int(os.environ.get("ROUNDS", "2"))):
    for lib in sys.argv[1:]:
        env = dict(os.environ)
        if lib != "main":
            env["AMC_LBA_LIB"] = os.path.abspath(lib)
        r = subprocess.run([sys.executable, "-c", CODE, WIN_FILE], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(lib, "failed:", r.stderr[-2000:])
            sys.exit(1)
        print(f"{lib:40s} {r.stdout.strip()}", flush=True)
