"""k_update's per-workgroup timeline (diagnostics, LBA_PHASE_TIMING): start / end of every workgroup (slots 14 / 15 of
the sweep's stamp rows), the GP pairs' publication (slot 13) and, with the fused evaluation, a tile's wait (slots 12 /
13), in us from the launch's first start.  python scripts/update_timeline.py [--config cfg1_local_50kf]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg1_local_50kf")
a = ap.parse_args()
path = os.path.join(ROOT, "gpurun_out", "update_timeline.bin")
os.environ["LBA_PHASE_TIMING"] = path
import amc_lba  # noqa: E402
from amc_lba.synth import make_config_window  # noqa: E402
from phase_times import load  # noqa: E402

w = make_config_window(a.config)
p = amc_lba.Problem(w, early_stop=0)
p.optimize(3)
p.close()
nt, lin, sch, shape, *_ = load(path)
st, en, pub, wt0, wt1 = lin[:, 14], lin[:, 15], lin[:, 13], lin[:, 12], lin[:, 11 + 2]
ok = st > 0
t0 = st[ok].min()
us = lambda v: (v - t0) / 100.0   # s_memrealtime: 100 MHz
print(f"k_update workgroups stamped: {ok.sum()} (of {nt} rows)")
print(f"  start: min 0  p50 {np.median(us(st[ok])):.2f}  max {us(st[ok]).max():.2f} us")
print(f"  end:   p50 {np.median(us(en[ok])):.2f}  p95 {np.percentile(us(en[ok]), 95):.2f}  max {us(en[ok]).max():.2f} us")
# the GP-pair workgroups come first (their rows have a publication stamp, slot 13, and no wait stamp after it)
gp = np.arange(nt) < int(os.environ.get("N_GP", "50"))
print(f"  GP pairs (first {gp.sum()} rows): start p50 {np.median(us(st[gp])):.2f}; published p50 {np.median(us(pub[gp])):.2f} "
      f"max {us(pub[gp]).max():.2f}; end p50 {np.median(us(en[gp])):.2f} max {us(en[gp]).max():.2f} us")
tl = ok & ~gp & (lin[:, 12] > t0)
if tl.any():
    print(f"  tiles: waiting from p50 {np.median(us(lin[tl, 12])):.2f}  max {us(lin[tl, 12]).max():.2f};  samples in p50 "
          f"{np.median(us(lin[tl, 13])):.2f}  max {us(lin[tl, 13]).max():.2f};  end p50 {np.median(us(en[tl])):.2f}  max "
          f"{us(en[tl]).max():.2f} us")
# the GP pairs' preparation phases (gp_pair_prep's stamps 0..5 in slots 5..10): pair chain (log / Ad), Jr^-1, w2 / A1,
# B1 / D, the sample poses + Jr (first chunk), the N blocks (last chunk)
names = ("log+Ad", "Jr^-1", "w2/A1", "B1/D", "samples", "N")
print("  GP pair prep stamps p50 (us): " + "  ".join(f"{n} {np.median(us(lin[gp, 5 + k])):.2f}" for k, n in enumerate(names)))
kb = np.arange(nt) == gp.sum()   # the first KF block (its end = its publication)
print(f"  KF block (row {gp.sum()}): start {us(st[kb]).max():.2f} end {us(en[kb]).max():.2f} us")
if tl.any():
    print(f"  tiles' back-substitution stamps: t_s done p50 {np.median(us(lin[tl, 5])):.2f}, landmarks done p50 "
          f"{np.median(us(lin[tl, 6])):.2f} max {us(lin[tl, 6]).max():.2f} us")
print(f"  KF block stamps: start {us(lin[kb, 5]).max():.2f}, trial states {us(lin[kb, 6]).max():.2f}, stored "
      f"{us(lin[kb, 7]).max():.2f}, published {us(lin[kb, 8]).max():.2f} us")
