"""lba_set_problem phases on a GPU box (LBA_SETUP_TIMING on stderr: host preprocessing, upload, solve
layout) and wall time, for repeated set-ups of one window on one engine (diagnostics)."""
import os
import sys
import time

os.environ["LBA_SETUP_TIMING"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "amc-slam_amd"))
import amc_lba  # noqa: E402
from amc_lba.synth import make_config_window  # noqa: E402

w = make_config_window(sys.argv[1] if len(sys.argv) > 1 else "cfg1_local_50kf")
p = amc_lba.Problem(w)
L = amc_lba.lib()
kfs, lm, obs, pri, vel, cams = p._keep
P = amc_lba.ptr
for _ in range(6):
    t0 = time.perf_counter()
    rc = L.lba_set_problem(p.h, P(kfs), len(kfs), P(lm), len(lm), P(obs), len(obs), P(pri), len(pri), P(vel), len(vel),
                           P(cams), len(cams))
    print(f"set_problem wall {1e3 * (time.perf_counter() - t0):.3f} ms rc {rc}", file=sys.stderr, flush=True)
