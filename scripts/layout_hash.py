"""Host layout fingerprints of lba_set_problem (lba_setup_host_profile: tiling, slab slots, device order; no GPU) for
the caller's LocalGPBA windows, configs 0-2 and three synthetic windows.  Run with two builds (or two values of
LBA_SETUP_THREADS) and compare the JSON files: the same layout, so bitwise the same LM runs.
    python scripts/layout_hash.py OUT.json"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "amc-slam_amd"))
import amc_lba  # noqa: E402
from amc_lba import mapsnap as ms  # noqa: E402
from amc_lba.synth import make_config_window, make_window  # noqa: E402

out = {}
m = ms.LocalGPBAMap(ms.make_map(n_kf=40, n_lm=8000, obs_per_lm=6, n_cam=4, seed=7))
for large in (False, True):
    for kf in (12, 20, 27, 33, 39):
        out[f"map_{int(large)}_{kf}"] = list(amc_lba.setup_host_profile(m.build_window(kf, large=large)[0])[1])
for c in ("cfg0_cpu_plumbing", "cfg1_local_50kf", "cfg2_global_500kf"):
    out[c] = list(amc_lba.setup_host_profile(make_config_window(c))[1])
for i, kw in enumerate((dict(n_opt_kf=6, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=1),
                        dict(n_opt_kf=99, n_fixed=1, n_lm=8000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=6),
                        dict(n_opt_kf=20, n_lm=5000, obs_per_lm=9, n_cam=4, gp=True, seed=11))):
    out[f"w{i}"] = list(amc_lba.setup_host_profile(make_window(**kw))[1])
json.dump({k: [int(x) for x in v] for k, v in out.items()}, open(sys.argv[1], "w"))
print(len(out), "layouts")
