"""Partitioned global BA (BASELINE config 4): landmark partitions of one window.

Every rank holds all keyframes (the same array, the same fixed flags), the landmarks l with
l % nranks == rank together with all of their observations, and rank 0 alone the motion-prior and
velocity edges.  The engine sums the ranks' reduced camera systems and trial sums every LM trial
(lba_set_partition*), so the keyframe states and LM decisions are identical on every rank, and each
rank back-substitutes its own landmarks (block_solver.hpp:461-482 per partition).
"""
import numpy as np

from .abi import PRIOR_DTYPE
from .synth import Window


def partition_window(win, rank, nranks):
    """The rank's share of `win`; returns (Window, landmark ids of the rank in `win`)."""
    if nranks <= 1:
        return win, np.arange(len(win.lm))
    lm_ids = np.arange(rank, len(win.lm), nranks)
    remap = -np.ones(len(win.lm), np.int64)
    remap[lm_ids] = np.arange(lm_ids.size)
    keep = remap[win.obs["lm"]] >= 0
    obs = win.obs[keep].copy()
    obs["lm"] = remap[obs["lm"]]
    priors = win.priors if rank == 0 else np.zeros(0, PRIOR_DTYPE)
    vel = win.vel_kfs if rank == 0 else np.zeros(0, np.int32)
    part = Window(kfs=win.kfs.copy(), lm=np.ascontiguousarray(win.lm[lm_ids]), obs=obs, priors=priors,
                  vel_kfs=np.ascontiguousarray(vel, dtype=np.int32), cams=win.cams.copy(), cfg=dict(win.cfg),
                  truth_lm=None if win.truth_lm is None else win.truth_lm[lm_ids],
                  name=f"{win.name}[{rank}/{nranks}]")
    return part, lm_ids
