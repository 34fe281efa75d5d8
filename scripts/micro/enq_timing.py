"""Host enqueue cost of queued trials (LBA_ENQ_TIMING) on the cfg1 window."""
import os, sys, time
os.environ["LBA_ENQ_TIMING"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
import amc_lba
from amc_lba.synth import make_config_window
win = make_config_window("cfg1_local_50kf")
p = amc_lba.Problem(win, device=0, early_stop=0)
for _ in range(4):
    t0 = time.perf_counter()
    n, st = p.optimize(10)
    print(f"optimize(10): {1e3 * (time.perf_counter() - t0):.2f} ms, {n} it", flush=True)
