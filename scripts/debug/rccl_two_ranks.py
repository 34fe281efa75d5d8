"""Rehearsal of the RCCL partition path with 2 ranks on ONE device (the multi-GPU run uses one
device per rank).  Bootstrap over gloo; each rank builds its landmark partition of a global-BA
window, joins the RCCL communicator through lba_set_partition_rccl and optimizes; rank 0 compares
with the unpartitioned problem.  Run: python -m torch.distributed.run --nproc-per-node 2
--master-addr 127.0.0.1 --master-port 29512 scripts/debug/rccl_two_ranks.py"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "amc-slam_amd")]
import amc_lba  # noqa: E402
from amc_lba.gba import partition_window  # noqa: E402
from amc_lba.synth import make_window  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
win = make_window(n_opt_kf=99, n_fixed=1, n_lm=8000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=6)
part, ids = partition_window(win, rank, world)
idt = torch.zeros(128, dtype=torch.uint8)
if rank == 0:
    idt.copy_(torch.frombuffer(bytearray(amc_lba.rccl_unique_id()), dtype=torch.uint8))
dist.broadcast(idt, 0)
p = amc_lba.Problem(part, device=0, early_stop=0, rccl_id=bytes(idt.numpy().tobytes()), rank=rank, nranks=world)
n, st = p.optimize(6)
kf, lm = p.state()
print(f"rank {rank}: iterations {n} trials {st.trials} chi2 {st.chi2_initial:.6f} -> {st.chi2_final:.6f}", flush=True)
t = torch.from_numpy(np.ascontiguousarray(kf["t"]).ravel().copy())
ts = [torch.zeros_like(t) for _ in range(world)]
dist.all_gather(ts, t)
if rank == 0:
    s = amc_lba.Problem(win, device=0, early_stop=0)
    n1, st1 = s.optimize(6)
    kf1, lm1 = s.state()
    same = all(torch.equal(ts[0], x) for x in ts)
    d = np.abs(kf["t"] - kf1["t"]).max() / np.abs(kf1["t"]).max()
    print(f"single: iterations {n1} trials {st1.trials} chi2 {st1.chi2_final:.6f}; ranks identical {same}; "
          f"kf rel diff {d:.2e}", flush=True)
    ok = same and n == n1 and st.trials == st1.trials and d < 1e-8 and abs(st.chi2_final - st1.chi2_final) <= 1e-9 * st1.chi2_final
    print("RCCL_TWO_RANKS", "OK" if ok else "MISMATCH", flush=True)
dist.barrier()
p.close()
dist.destroy_process_group()
