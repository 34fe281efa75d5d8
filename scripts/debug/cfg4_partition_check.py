"""Config 4: single problem vs 2- and 3-rank partitions (in-process group), per LM iteration count."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "amc-slam_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import numpy as np
from amc_lba import Problem
from amc_lba.synth import make_config_window
from test_gpu_partition import run_partitioned

win = make_config_window("cfg4_global_5k")
for iters in (1, 2):
    p = Problem(win, early_stop=0)
    n, st = p.optimize(iters)
    kf, lm = p.state()
    p.close()
    print(f"iters {iters}: single chi2 {st.chi2_initial:.10e} -> {st.chi2_final:.10e} trials {st.trials}", flush=True)
    for nr in (2, 3):
        res, kfs, lm_p = run_partitioned(win, nr, iters)
        n_r, st_r = res[0]
        dt = np.abs(kfs[0]["t"] - kf["t"]).max() / np.abs(kf["t"]).max()
        dl = np.abs(lm_p - lm).max() / np.abs(lm).max()
        print(f"   {nr} ranks: chi2 {st_r.chi2_initial:.10e} -> {st_r.chi2_final:.10e} trials {st_r.trials} "
              f"rel dt {dt:.2e} rel dlm {dl:.2e}", flush=True)
