"""Diagnostics: queued vs host-driven LM loop, and run-to-run determinism of each, on the small
parity windows (prints the first differing quantity)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
import numpy as np
from amc_lba import Problem
from amc_lba.abi import FLAG_HOST_LOOP
from amc_lba.synth import make_window
WINDOWS = {   # the small windows of tests/test_gpu_parity.py
    "gp_small": dict(n_opt_kf=6, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=1),
    "gp_stereo": dict(n_opt_kf=5, n_lm=250, obs_per_lm=6, n_cam=3, gp=True, stereo_frac=1.0, seed=2),
    "mono_only": dict(n_opt_kf=9, n_fixed=1, n_lm=400, obs_per_lm=5, n_cam=1, gp=False, seed=3),
    "two_fixed": dict(n_opt_kf=6, n_fixed=2, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=4),
    "global_shape": dict(n_opt_kf=11, n_fixed=1, n_lm=500, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=5),
}


def run(win, flags, es, iters):
    p = Problem(win, early_stop=es, flags=flags)
    out = []
    for it in iters:
        n, st = p.optimize(it)
        kf, lm = p.state()
        out.append((n, st.iterations, st.trials, st.result, st.solve_failures, st.chi2_initial, st.chi2_final,
                    st.lambda_final, kf["t"].copy(), lm.copy()))
    p.close()
    return out


def cmp(a, b):
    for k, (x, y) in enumerate(zip(a, b)):
        for f, (u, v) in enumerate(zip(x, y)):
            eq = np.array_equal(u, v) if isinstance(u, np.ndarray) else u == v
            if not eq:
                d = np.abs(u - v).max() if isinstance(u, np.ndarray) else abs(u - v)
                return f"call {k} field {f}: diff {d:.3e}"
    return "equal"


for name in WINDOWS:
    win = make_window(**WINDOWS[name])
    for es in (1, 0):
        q1 = run(win, 0, es, (25, 3))
        q2 = run(win, 0, es, (25, 3))
        h1 = run(win, FLAG_HOST_LOOP, es, (25, 3))
        h2 = run(win, FLAG_HOST_LOOP, es, (25, 3))
        print(f"{name:13s} es={es} queued-rerun: {cmp(q1, q2):28s} host-rerun: {cmp(h1, h2):28s} "
              f"queued-vs-host: {cmp(q1, h1)}", flush=True)
        for k in range(1, 25):   # first iteration count at which the modes differ
            a = run(win, 0, es, (k,))
            b = run(win, FLAG_HOST_LOOP, es, (k,))
            if cmp(a, b) != "equal":
                print(f"   first differs after {k} iterations: {cmp(a, b)}; trials {a[0][2]} vs {b[0][2]}", flush=True)
                break
