"""Bitwise comparison of two LocalGPBA adapter builds (the in-tree one = "main", or a path): LocalGPBA for keyframes
20..39 in mapping order on a fresh synthetic map, normal and bLarge, then bExtrinsic; hashes of every call's result
counters and of the map snapshot after each sequence.  GPU run.
    python scripts/cmp_map_libs.py main amc-slam_amd/lib/exp/map_head.so"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import hashlib, sys
sys.path.insert(0, %r)
from amc_lba import mapsnap as ms
snap = ms.make_map(n_kf=40, n_lm=8000, obs_per_lm=6, n_cam=4, seed=7)
out = []
for large, extr in ((False, False), (True, False), (False, True)):
    m = ms.LocalGPBAMap(snap)
    h = hashlib.sha256()
    for kf in range(20, 40):
        rc, r = m.local_gpba(kf, large=large, extrinsic=extr)
        h.update(repr((rc, r.status, r.n_mp, r.n_erased_gp, r.n_erased, r.n_set_bad, r.iterations, r.chi2_initial,
                       r.chi2_final)).encode())
    h.update(ms.pack(m.save()))
    m.close()
    out.append(h.hexdigest()[:16])
print(" ".join(out))
""" % os.path.join(ROOT, "amc-slam_amd")
res = {}
for lib in sys.argv[1:]:
    env = dict(os.environ)
    if lib != "main":
        env["AMC_LBA_MAP_LIB"] = os.path.abspath(lib)
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=600)
    if r.returncode:
        print(lib, "failed:", r.stderr[-2000:])
        sys.exit(1)
    res[lib] = r.stdout.split()
    print(lib, res[lib], flush=True)
vals = list(res.values())
print("bitwise identical" if all(v == vals[0] for v in vals) else "DIFFERENT")
sys.exit(0 if all(v == vals[0] for v in vals) else 1)
