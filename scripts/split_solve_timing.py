"""Distributed factorisation (LBA_FLAG_SUBTREE_SOLVE) on one GPU: the window of a config split over N ranks of
an in-process group (lba_partition_assign) against the unpartitioned problem.  Per rank: LM iterations, chi2,
the solve's device time per trial (k_chol_flow launches + the top all-reduce between them, LBA_FLAG_TIME_SWEEP),
the split (panels in the rank's subtree / the top); the gathered state against the unpartitioned one.  On one
GPU the ranks' kernels share the chip, so the per-rank times are an upper bound of a one-GPU-per-rank run.

    python scripts/split_solve_timing.py [--config cfg2_global_500kf] [--ranks 2] [--iters 5]
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
import amc_lba  # noqa: E402
from amc_lba import Group, Problem  # noqa: E402
from amc_lba.abi import FLAG_BAND_SOLVE, FLAG_SUBTREE_SOLVE, FLAG_TIME_SWEEP  # noqa: E402
from amc_lba.gba import partition_window  # noqa: E402
from amc_lba.synth import make_config_window  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2_global_500kf")
ap.add_argument("--ranks", type=int, default=2)
ap.add_argument("--iters", type=int, default=5)
args = ap.parse_args()
win = make_config_window(args.config)
t0 = time.time()
p = Problem(win, early_stop=0, flags=FLAG_BAND_SOLVE | FLAG_TIME_SWEEP)
n1, st1 = p.optimize(args.iters)
kf1, lm1 = p.state()
info1 = p.solver_info()
p.close()
print(f"{args.config}: single problem  iters {n1} trials {st1.trials} chi2 {st1.chi2_initial:.6e} -> {st1.chi2_final:.6e}  "
      f"solve {st1.ms_k_solve / max(st1.n_k_solve, 1) * 1e3:8.1f} us/trial  sweep "
      f"{st1.ms_k_linearize / max(st1.n_k_linearize, 1) * 1e3:8.1f} us  solver {info1}  ({time.time() - t0:.1f} s)", flush=True)
N = args.ranks
assign = amc_lba.partition_assign(win, N)
print(f"split over {N}: panels {assign[3].tolist()} (system, top, largest subtree); landmarks per rank "
      f"{np.bincount(assign[0], minlength=N).tolist()}", flush=True)
parts = [partition_window(win, r, N, assign) for r in range(N)]
g = Group(N)
probs, res = [None] * N, [None] * N


def run(fn):
    ts = [threading.Thread(target=fn, args=(r,)) for r in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


run(lambda r: probs.__setitem__(r, Problem(parts[r][0], group=g, rank=r, early_stop=0,
                                           flags=FLAG_SUBTREE_SOLVE | FLAG_TIME_SWEEP)))
run(lambda r: res.__setitem__(r, probs[r].optimize(args.iters)))
own = probs[0].kf_owner()
kf = probs[0].state()[0].copy()
lm = np.zeros_like(win.lm)
for r in range(N):
    kr, lr = probs[r].state()
    kf[own == r] = kr[own == r]
    lm[parts[r][1]] = lr
    n, st = res[r]
    print(f"  rank {r}: iters {n} trials {st.trials} chi2 {st.chi2_final:.6e}  solve "
          f"{st.ms_k_solve / max(st.n_k_solve, 1) * 1e3:8.1f} us/trial  sweep "
          f"{st.ms_k_linearize / max(st.n_k_linearize, 1) * 1e3:8.1f} us  keyframes owned {(own == r).sum()} "
          f"(top {(own < 0).sum()})  device MB {probs[r].device_bytes() / 2**20:.0f}", flush=True)
    si = probs[r].split_info()
    print(f"          factorisation GFLOP {si['rank_flops'] / 1e9:.3f} of {si['system_flops'] / 1e9:.3f} "
          f"({si['rank_flops'] / si['system_flops']:.2f}); all-reduce per trial {si['allreduce_bytes'] / 2**20:.2f} MB "
          f"(replicated solve {si['replicated_allreduce_bytes'] / 2**20:.1f} MB); panels own {si['own_panels']:.0f} "
          f"top {si['top_panels']:.0f}", flush=True)
for q in probs:
    q.close()
g.close()
dt = np.abs(kf["t"] - kf1["t"]).max() / np.abs(kf1["t"]).max()
dl = np.abs(lm - lm1).max() / np.abs(lm1).max()
print(f"  gathered state vs single: keyframe t rel {dt:.2e}, landmarks rel {dl:.2e}; same iterations / trials: "
      f"{all(r[0] == n1 and r[1].trials == st1.trials for r in res)}", flush=True)
