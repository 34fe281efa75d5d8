"""Host preprocessing of lba_set_problem alone (lba_setup_host_profile: no device), per phase, median of
repeats, for a config window; run once per LBA_SETUP_THREADS value to see the threaded phases scale.

    python scripts/setup_profile.py [--config cfg1_local_50kf] [--reps 9]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if os.environ.get("_SETUP_PROFILE_CHILD"):
    sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
    import numpy as np
    import amc_lba
    from amc_lba.synth import make_config_window
    cfg, reps = sys.argv[1], int(sys.argv[2])
    w = make_config_window(cfg)
    r = np.array([amc_lba.setup_host_profile(w)[0] for _ in range(reps)])
    med = np.median(r, axis=0)
    print(f"threads {os.environ.get('LBA_SETUP_THREADS', 'auto'):>4}: order/pairs {med[0]:7.3f} ms  tiles {med[1]:7.3f} ms  "
          f"slots/state {med[2]:7.3f} ms  total {np.median(r.sum(1)):7.3f} ms", flush=True)
    sys.exit(0)

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg1_local_50kf")
ap.add_argument("--reps", type=int, default=9)
args = ap.parse_args()
for th in ("1", "2", "4", "8"):
    env = dict(os.environ, _SETUP_PROFILE_CHILD="1", LBA_SETUP_THREADS=th)
    subprocess.run([sys.executable, os.path.abspath(__file__), args.config, str(args.reps)], env=env, check=True)
