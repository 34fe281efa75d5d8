"""The LM of the caller's LocalGPBA windows alone (for rocprofv3 --kernel-trace --stats): the windows of keyframes
20..39 of a synthetic 40-keyframe, 4-camera map (normal, or bLarge with --large), set up on one engine in turn, each
optimised for 10 iterations; prints the median ms per optimize(10).  GPU run.
    python scripts/map_window_lm.py [--large] [--passes 3]"""
import argparse
import os
import pickle
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--large", action="store_true")
ap.add_argument("--passes", type=int, default=3)
args = ap.parse_args()
# the windows come from the adapter in a process of its own (this process loads one engine library only)
f = os.path.join(os.environ.get("TMPDIR", "/tmp"), "map_window_lm.pkl")
subprocess.run([sys.executable, "-c", (
    "import sys, pickle; sys.path.insert(0, %r)\n"
    "from amc_lba import mapsnap as ms\n"
    "m = ms.LocalGPBAMap(ms.make_map(n_kf=40, n_lm=8000, obs_per_lm=6, n_cam=4, seed=7))\n"
    "pickle.dump([m.build_window(kf, large=%r)[0] for kf in range(20, 40)], open(%r, 'wb'))\n")
    % (os.path.join(ROOT, "amc-slam_amd"), args.large, f)], check=True, timeout=300)
wins = pickle.load(open(f, "rb"))
import amc_lba  # noqa: E402
p = amc_lba.Problem(wins[0])
t, it = [], []
for _ in range(args.passes):
    for W in wins:
        p.set_window(W)
        t0 = time.perf_counter()
        n, st = p.optimize(10)
        t.append(time.perf_counter() - t0)
        it.append(st.trials)
p.close()
print(f"optimize(10) median {np.median(t) * 1e3:.3f} ms, trials mean {np.mean(it):.2f}, windows {len(wins)}, "
      f"obs mean {np.mean([len(W.obs) for W in wins]):.0f}")
