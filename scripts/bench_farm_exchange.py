"""Cost of one window-boundary exchange (lba_farm_exchange) on one GPU, the collective stubbed.

Rank 1 of a config-1 farm of two windows (stride 25: ~50 % shared): its problem is planned with a stub
all-reduce (returns at once, so the exchange buffer holds rank 1's own slot and zeros), then
lba_farm_exchange runs back to back.  Prints the host wall time per exchange (launches + stream sync)
and the plan's counts; under rocprofv3 --kernel-trace --stats the two kernels' device times show.

    python scripts/bench_farm_exchange.py [--reps 200]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))

import numpy as np  # noqa: E402

import amc_lba  # noqa: E402
from amc_lba import farm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=200)
ap.add_argument("--config", default="cfg1_local_50kf")
args = ap.parse_args()

wins, infos = farm.make_farm_windows(args.config, 2, seed=20250912, stride=25)
import threading  # noqa: E402

import torch  # noqa: E402

# (1) rank 0 alone with a stub collective: the publishing side (pack kernel only; nothing to receive)
prob = amc_lba.Problem(wins[0], early_stop=0)
STUB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p)
stub = STUB(lambda buf, n, stream, user: 0)
L = amc_lba.lib()
prob._check(L.lba_set_farm(prob.h, 0, 2, ctypes.cast(stub, ctypes.c_void_p), None))
kfo, lmo = farm.publish_owners(infos[0])
print("rank 0 plan (kf pub, lm pub, kf recv, lm recv, unmatched):",
      prob.farm_plan(wins[0].kf_gid, kfo, wins[0].lm_gid, lmo), flush=True)
for _ in range(10):
    prob.farm_exchange()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.reps):
    prob.farm_exchange()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / args.reps
print(f"stub collective, publishing rank: {dt * 1e6:.1f} us per boundary (host wall incl. launches)", flush=True)
prob.close()

# (2) both windows on this GPU, the in-process group as the collective (its sum kernel is the
#     all-gather): pack, gather, unpack; the two ranks run from two threads in lockstep
g = amc_lba.Group(2)
probs = [amc_lba.Problem(w, early_stop=0) for w in wins]
for r, p in enumerate(probs):
    p.set_farm_group(g, r)
cnt = [None, None]


def run(r, fn):
    ts = [threading.Thread(target=fn, args=(q,)) for q in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


run(0, lambda r: cnt.__setitem__(r, probs[r].farm_plan(wins[r].kf_gid, farm.publish_owners(infos[r])[0],
                                                       wins[r].lm_gid, farm.publish_owners(infos[r])[1])))
print("group plans:", cnt, flush=True)


def reps(r):
    for _ in range(args.reps):
        probs[r].farm_exchange()
    torch.cuda.synchronize()


run(0, lambda r: [probs[r].farm_exchange() for _ in range(10)])
torch.cuda.synchronize()
t0 = time.perf_counter()
run(0, reps)
dt = (time.perf_counter() - t0) / args.reps
print(f"in-process group, both ranks: {dt * 1e6:.1f} us per boundary (host wall, two threads)", flush=True)
for p in probs:
    n, st = p.optimize(2)
    print(f"optimize after exchanges: {n} iterations, chi2 {st.chi2_initial:.6e} -> {st.chi2_final:.6e}")
    p.close()
g.close()
