"""One damped solve on a small GP window; prints the factorisation status on failure (diagnostics)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "amc-slam_amd"))
import amc_lba
from amc_lba.synth import make_window
w = make_window(n_opt_kf=int(sys.argv[1]) if len(sys.argv) > 1 else 6, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=1)
p = amc_lba.Problem(w)
p.linearize()
rc = amc_lba.lib().lba_solve_step(p.h, 1.0, None)
print("rc", rc, amc_lba.lib().lba_last_error(p.h).decode(), "solver", p.solver_info())
