"""Tracking-side pose optimisation throughput (lba_track, one workgroup per frame): frames/s and
latency per launch for batches of 1 .. 512 frames, next to the oracle (orc_track_pose, 1 CPU thread)
on a few frames of the same kind.  Frames: KF k of a 4-camera window (~1.2-1.8k edges each)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "amc-slam_amd"), os.path.join(ROOT, "oracle")]
from amc_lba.synth import make_window  # noqa: E402
from amc_lba.track import TRACK_FRAME_DTYPE, TRACK_OBS_DTYPE, Tracker, make_track_frames, track_config  # noqa: E402

win = make_window(n_opt_kf=40, n_fixed=1, n_lm=10000, obs_per_lm=6, n_cam=4, gp=True, seed=11, perturb=False)
base_f, base_o = make_track_frames(win, list(range(3, 38)), fix_prev=True, seed=3)


def batch(n):
    fr = np.zeros(n, TRACK_FRAME_DTYPE)
    obs = []
    off = 0
    for i in range(n):
        j = i % len(base_f)
        fr[i] = base_f[j]
        o = base_o[base_f[j]["obs0"]: base_f[j]["obs0"] + base_f[j]["n_obs"]]
        fr[i]["obs0"] = off
        off += len(o)
        obs.append(o)
    return fr, np.concatenate(obs).astype(TRACK_OBS_DTYPE)


cfg = track_config()
t = Tracker(cfg)
out = {"workload": "tracking frames (PoseGPOptimizationFromeLastFrame), 4 cameras, prev fixed",
       "edges_per_frame_mean": float(base_f["n_obs"].mean())}
res = []
for n in (1, 8, 64, 256, 512):
    fr, ob = batch(n)
    t.track(fr.copy(), ob.copy(), win.cams)   # warm-up
    reps = 5 if n <= 64 else 2
    t0 = time.perf_counter()
    for _ in range(reps):
        t.track(fr.copy(), ob.copy(), win.cams)
    dt = (time.perf_counter() - t0) / reps
    res.append({"frames": n, "ms_per_launch": dt * 1e3, "frames_per_s": n / dt})
    print(json.dumps(res[-1]), flush=True)
out["gpu"] = res
if "--no-cpu" not in sys.argv:
    import orc
    t0 = time.perf_counter()
    for j in range(4):
        a = base_f[j:j + 1].copy()
        o = base_o[base_f[j]["obs0"]: base_f[j]["obs0"] + base_f[j]["n_obs"]].copy()
        orc.track_pose(cfg, a, o, win.cams)
    dt = (time.perf_counter() - t0) / 4
    out["cpu_baseline"] = {"frames_per_s": 1.0 / dt, "cores": 1, "kind": "port",
                           "sample": "4 frames, oracle/lba_oracle.c orc_track_pose (-O3, 1 thread)"}
print(json.dumps(out), flush=True)
