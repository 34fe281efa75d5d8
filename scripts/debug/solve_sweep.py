"""Per-trial solve time, L^-1 (dense) vs substitution (band), over global-BA window sizes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "amc-slam_amd")]
import amc_lba  # noqa: E402
from amc_lba.abi import FLAG_BAND_SOLVE, FLAG_DENSE_SOLVE, FLAG_TIME_PHASES  # noqa: E402
from amc_lba.synth import make_window  # noqa: E402

for nkf in (50, 100, 150, 200, 300, 500):
    win = make_window(n_opt_kf=nkf - 1, n_fixed=1, n_lm=400 * nkf, obs_per_lm=6, n_cam=4, gp=True, global_ba=True,
                      seed=3)
    out = []
    for name, fl in (("dense", FLAG_DENSE_SOLVE), ("band", FLAG_BAND_SOLVE)):
        p = amc_lba.Problem(win, early_stop=0, flags=FLAG_TIME_PHASES | fl)
        p.optimize(2)
        n, st = p.optimize(10)
        out.append(f"{name} {st.ms_solve / max(st.trials, 1):.3f} ms/trial")
        p.close()
    print(nkf, (nkf - 1) * 12 // 32 + 1, "panels:", ", ".join(out), flush=True)
