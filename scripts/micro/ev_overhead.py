"""A/B: LM iterations/s of the cfg1 window with and without the per-iteration sweep events."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
import torch
import amc_lba
from amc_lba.synth import make_config_window
win = make_config_window("cfg1_local_50kf")
for rep in range(2):
    for flags in (0, amc_lba.abi.FLAG_TIME_SWEEP, amc_lba.abi.FLAG_HOST_LOOP):
        p = amc_lba.Problem(win, device=0, early_stop=0, flags=flags)
        p.optimize(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for _ in range(4):
            k, st = p.optimize(10)
            n += k
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"flags={flags} iters={n} it/s={n / dt:.1f}", flush=True)
        p.close()
