"""Run LocalGPBA through the C++ adapter on the GPU and dump the map before/after (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "amc-slam_amd")]
from amc_lba import mapsnap as ms  # noqa: E402

kf_id, large = int(sys.argv[1]), bool(int(sys.argv[2]))
s = ms.make_map(n_kf=30, n_lm=3000, obs_per_lm=5, n_cam=4, seed=7)
m = ms.LocalGPBAMap(s)
rc, res = m.local_gpba(kf_id, large=large)
print("rc", rc, res.iterations, res.chi2_initial, res.chi2_final, res.n_erased, res.n_erased_gp)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
open(os.path.join(ROOT, "gpurun_out", f"adapter_{kf_id}_{int(large)}.snap"), "wb").write(ms.pack(m.save()))
