"""Partitioned global BA (BASELINE config 4): landmark partitions of one window.

Every rank holds all keyframes (the same array, the same fixed flags) and a share of the landmarks with
all of their observations, and of the motion-prior / velocity edges.  Two splits:

- replicated solve (lba_set_partition): landmark l on rank l % nranks, every edge on rank 0; the engine
  sums the ranks' whole reduced camera systems every LM trial and every rank factors all of it;
- distributed factorisation (LBA_FLAG_SUBTREE_SOLVE): lba_partition_assign cuts the nested dissection of
  the reduced system into one subtree per rank plus the top separators and gives each landmark / edge to
  the rank whose subtree holds its keyframes; a rank factors its subtree alone, the ranks sum only their
  contributions to the top (tiles and right-hand side), and every rank factors the top.

In both the keyframe states of the top and the LM decisions are identical on every rank, and each rank
back-substitutes its own landmarks (block_solver.hpp:461-482 per partition); with the distributed
factorisation a keyframe of a rank's subtree is up to date on that rank only (lba_kf_owner).
"""
import numpy as np

from .abi import PRIOR_DTYPE
from .synth import Window


def partition_window(win, rank, nranks, assign=None):
    """The rank's share of `win`; returns (Window, landmark ids of the rank in `win`).  assign: (lm_rank,
    prior_rank, vel_rank) from amc_lba.partition_assign (distributed factorisation), or None for the
    replicated solve's split (l % nranks, edges on rank 0)."""
    if nranks <= 1:
        return win, np.arange(len(win.lm))
    if np.any(np.asarray(win.cams["ext_free"]) != 0):
        # a partitioned lba_set_problem rejects free extrinsics (LBA_E_LIMIT), and lba_partition_assign, which sees no
        # cameras, plans the keyframe-only pattern: refuse the split up front rather than fail later on some rank
        raise ValueError("partition_window: free extrinsics (lba_cam.ext_free) are not supported in a partitioned "
                         "problem; optimise the extrinsic pass (bExtrinsic) on one GPU")
    if assign is None:
        lm_ids = np.arange(rank, len(win.lm), nranks)
        pri_keep = np.full(len(win.priors), rank == 0)
        vel_keep = np.full(len(win.vel_kfs), rank == 0)
    else:
        lm_rank, pri_rank, vel_rank = assign[:3]
        lm_ids = np.nonzero(np.asarray(lm_rank) == rank)[0]
        pri_keep = np.asarray(pri_rank) == rank
        vel_keep = np.asarray(vel_rank) == rank
    remap = -np.ones(len(win.lm), np.int64)
    remap[lm_ids] = np.arange(lm_ids.size)
    keep = remap[win.obs["lm"]] >= 0
    obs = win.obs[keep].copy()
    obs["lm"] = remap[obs["lm"]]
    priors = win.priors[pri_keep] if len(win.priors) else np.zeros(0, PRIOR_DTYPE)
    vel = np.asarray(win.vel_kfs)[vel_keep] if len(win.vel_kfs) else np.zeros(0, np.int32)
    part = Window(kfs=win.kfs.copy(), lm=np.ascontiguousarray(win.lm[lm_ids]), obs=obs,
                  priors=np.ascontiguousarray(priors), vel_kfs=np.ascontiguousarray(vel, dtype=np.int32),
                  cams=win.cams.copy(), cfg=dict(win.cfg),
                  truth_lm=None if win.truth_lm is None else win.truth_lm[lm_ids],
                  name=f"{win.name}[{rank}/{nranks}]")
    return part, lm_ids
