"""lba_set_problem of one config window, set up twice on one engine (the second on warm buffers): wall ms and phases
per set-up.  Under rocprofv3 --kernel-trace --stats it also gives the set-up's kernels (k_zero_ranges, k_gp_prep).
GPU run; AMC_LBA_LIB selects another build.
    python scripts/setup_time_cfg.py [--config cfg4_global_5k]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "amc-slam_amd"))
import amc_lba  # noqa: E402
from amc_lba.synth import make_config_window  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg4_global_5k")
a = ap.parse_args()
W = make_config_window(a.config)
print(f"window ready: {len(W.obs)} observations", flush=True)
t = time.perf_counter()
p = amc_lba.Problem(W)
t1 = time.perf_counter() - t
ph1 = p.setup_phases()
t = time.perf_counter()
p.set_window(W)
t2 = time.perf_counter() - t
ph2 = p.setup_phases()
print(f"{a.config}: set-up {t1 * 1e3:.1f} ms (cold) {ph1}; {t2 * 1e3:.1f} ms (warm) {ph2}", flush=True)
p.close()
