"""Multi-GPU local-BA window farm (BASELINE config 3).

Local BA shards at the window level: every rank (one process per GPU) owns one LocalGPBA-shaped
window (50 optimisable KFs) cut from the same trajectory, neighbouring windows overlap by
`stride` keyframes, so they share keyframes and landmarks.  During LM there is no exchange at
all; at each window boundary the owner of every shared vertex (the lowest rank whose window
contains it, computed identically on every rank from the deterministic window layout) publishes
its estimate with ONE all_gather of a fixed-size fp64 buffer, and the other ranks overwrite their
copies.  Over RCCL this is a single ring all_gather of ~0.3 MB per rank on xGMI.
"""
from dataclasses import dataclass

import numpy as np

from .synth import CONFIGS, cut_window, make_window

_MAP_CACHE = {}


def global_map(config, world, seed, stride):
    key = (config, world, seed, stride)
    if key not in _MAP_CACHE:
        kw = dict(CONFIGS[config])
        n_opt = kw["n_opt_kf"]
        n_total = stride * (world - 1) + n_opt + 1
        kw["n_lm"] = int(round(kw["n_lm"] * n_total / (n_opt + 1)))
        kw["n_opt_kf"] = n_total - 1
        kw["n_fixed"] = 1
        _MAP_CACHE[key] = make_window(seed=seed, name=f"{config}-map", **kw)
    return _MAP_CACHE[key]


@dataclass
class SharedInfo:
    lm_owner: np.ndarray      # per local landmark: owning rank
    kf_owner: np.ndarray      # per local keyframe: owning rank
    lm_shared: np.ndarray     # per local landmark: appears in >= 2 windows
    kf_shared: np.ndarray
    max_lm_owned: int         # max over ranks of owned shared landmarks (all_gather buffer rows)
    max_kf_owned: int


def farm_layout(windows):
    """Ownership of shared vertices for a list of windows (identical on every rank)."""
    lm_first, lm_count, kf_first, kf_count = {}, {}, {}, {}
    for r, w in enumerate(windows):
        for g in w.lm_gid.tolist():
            lm_first.setdefault(g, r)
            lm_count[g] = lm_count.get(g, 0) + 1
        for g in w.kf_gid.tolist():
            kf_first.setdefault(g, r)
            kf_count[g] = kf_count.get(g, 0) + 1
    infos = []
    for r, w in enumerate(windows):
        lo = np.array([lm_first[g] for g in w.lm_gid.tolist()])
        ko = np.array([kf_first[g] for g in w.kf_gid.tolist()])
        ls = np.array([lm_count[g] > 1 for g in w.lm_gid.tolist()])
        ks = np.array([kf_count[g] > 1 for g in w.kf_gid.tolist()])
        infos.append((lo, ko, ls, ks))
    max_lm = max(int(((lo == r) & ls).sum()) for r, (lo, _, ls, _) in enumerate(infos))
    max_kf = max(int(((ko == r) & ks).sum()) for r, (_, ko, _, ks) in enumerate(infos))
    return [SharedInfo(lo, ko, ls, ks, max(max_lm, 1), max(max_kf, 1)) for lo, ko, ls, ks in infos]


def make_farm_windows(config, world, seed=20250912, stride=25):
    g = global_map(config, world, seed, stride)
    n_opt = CONFIGS[config]["n_opt_kf"]
    wins = [cut_window(g, r * stride, n_opt, name=f"{config}-w{r}") for r in range(world)]
    return wins, farm_layout(wins)


def make_rank_window(config, rank, world, seed=20250912, stride=25):
    wins, infos = make_farm_windows(config, world, seed, stride)
    return wins[rank], infos[rank]


class SharedExchange:
    """Window-boundary exchange of shared landmark / keyframe estimates (torch.distributed)."""

    def __init__(self, win, info, rank, world, device=None, group=None):
        import torch
        self.torch = torch
        self.win, self.info, self.rank, self.world = win, info, rank, world
        self.device = device if device is not None else torch.device("cpu")
        self.group = group
        self.lm_send = np.nonzero((info.lm_owner == rank) & info.lm_shared)[0]
        self.lm_recv = np.nonzero(info.lm_owner != rank)[0]
        self.kf_send = np.nonzero((info.kf_owner == rank) & info.kf_shared)[0]
        self.kf_recv = np.nonzero(info.kf_owner != rank)[0]
        self.lm_gid_to_local = {int(g): i for i, g in enumerate(win.lm_gid)}
        self.kf_gid_to_local = {int(g): i for i, g in enumerate(win.kf_gid)}
        self.bytes_per_exchange = 8 * (info.max_lm_owned * 4 + info.max_kf_owned * 14) * world

    def _pack(self, lm, kfs):
        torch = self.torch
        L = np.full((self.info.max_lm_owned, 4), -1.0)
        L[: self.lm_send.size, 0] = self.win.lm_gid[self.lm_send]
        L[: self.lm_send.size, 1:] = lm[self.lm_send]
        K = np.full((self.info.max_kf_owned, 14), -1.0)
        K[: self.kf_send.size, 0] = self.win.kf_gid[self.kf_send]
        K[: self.kf_send.size, 1:5] = kfs["q"][self.kf_send]
        K[: self.kf_send.size, 5:8] = kfs["t"][self.kf_send]
        K[: self.kf_send.size, 8:14] = kfs["vel"][self.kf_send]
        buf = np.concatenate([L.ravel(), K.ravel()])
        return torch.from_numpy(buf).to(self.device)

    def exchange(self, prob):
        """prob: anything with state() -> (kfs, lm) and set_state(kfs=, lm=) (amc_lba.Problem)."""
        torch = self.torch
        import torch.distributed as dist
        kfs, lm = prob.state()
        send = self._pack(lm, kfs)
        gathered = [torch.empty_like(send) for _ in range(self.world)]
        dist.all_gather(gathered, send, group=self.group)
        nL = self.info.max_lm_owned * 4
        lm_new, kfs_new = lm.copy(), kfs.copy()
        for r, t in enumerate(gathered):
            if r == self.rank:
                continue
            a = t.cpu().numpy()
            L = a[:nL].reshape(-1, 4)
            K = a[nL:].reshape(-1, 14)
            for row in L[L[:, 0] >= 0]:
                i = self.lm_gid_to_local.get(int(row[0]))
                if i is not None and self.info.lm_owner[i] == r:
                    lm_new[i] = row[1:]
            for row in K[K[:, 0] >= 0]:
                i = self.kf_gid_to_local.get(int(row[0]))
                if i is not None and self.info.kf_owner[i] == r:
                    kfs_new[i]["q"] = row[1:5]
                    kfs_new[i]["t"] = row[5:8]
                    kfs_new[i]["vel"] = row[8:14]
        prob.set_state(kfs=kfs_new, lm=lm_new)
        return lm_new, kfs_new
