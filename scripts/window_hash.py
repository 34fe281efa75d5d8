"""Digests of the flat windows the LocalGPBA / BundleAdjustment adapters build (no GPU): LocalGPBA windows (normal and
bLarge) for keyframes 5.. of two synthetic maps, plus each map's global-BA window.  Run with two adapter builds
(AMC_LBA_MAP_LIB selects another one) and compare the JSON files: a byte-identical window build.
    python scripts/window_hash.py OUT.json"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "amc-slam_amd"))
from amc_lba import mapsnap as ms  # noqa: E402


def digest(W, *extra):
    h = hashlib.sha256()
    for a in (W.kfs, W.lm, W.obs, W.priors, W.vel_kfs, W.cams) + extra:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


out = {}
for seed, nkf in ((7, 40), (3, 30)):
    m = ms.LocalGPBAMap(ms.make_map(n_kf=nkf, n_lm=6000, obs_per_lm=6, n_cam=4, seed=seed))
    for large in (False, True):
        for kf in range(5, nkf):
            W, kid, mid, tag = m.build_window(kf, large=large)
            out[f"{seed}_{int(large)}_{kf}"] = digest(W, kid, mid, tag)
    W, kid, mid, tag = m.build_ba_window()
    out[f"{seed}_ba"] = digest(W, kid, mid, tag)
json.dump(out, open(sys.argv[1], "w"))
print(len(out), "windows")
