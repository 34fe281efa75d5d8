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
    """config: a CONFIGS name or a make_window keyword dict (its per-window shape)."""
    ckey = config if isinstance(config, str) else tuple(sorted(config.items()))
    key = (ckey, world, seed, stride)
    if key not in _MAP_CACHE:
        kw = dict(CONFIGS[config] if isinstance(config, str) else config)
        n_opt = kw["n_opt_kf"]
        n_total = stride * (world - 1) + n_opt + 1
        kw["n_lm"] = int(round(kw["n_lm"] * n_total / (n_opt + 1)))
        kw["n_opt_kf"] = n_total - 1
        kw["n_fixed"] = 1
        _MAP_CACHE[key] = make_window(seed=seed, name=f"{ckey}-map" if isinstance(ckey, str) else "farm-map", **kw)
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
    n_opt = (CONFIGS[config] if isinstance(config, str) else config)["n_opt_kf"]
    tag = config if isinstance(config, str) else "farm"
    wins = [cut_window(g, r * stride, n_opt, name=f"{tag}-w{r}") for r in range(world)]
    return wins, farm_layout(wins)


def make_rank_window(config, rank, world, seed=20250912, stride=25):
    wins, infos = make_farm_windows(config, world, seed, stride)
    return wins[rank], infos[rank]


def publish_owners(info):
    """Owner arrays in the C ABI's convention (include/amc_lba.h, lba_farm_plan): the publishing rank of
    every shared vertex, -1 for a vertex no other window holds."""
    kf = np.where(info.kf_shared, info.kf_owner, -1).astype(np.int32)
    lm = np.where(info.lm_shared, info.lm_owner, -1).astype(np.int32)
    return kf, lm


class DeviceExchange:
    """Window-boundary exchange through the engine (lba_farm_plan / lba_farm_exchange): pack kernel,
    all-gather over the problem's collective (RCCL or an in-process group), unpack kernel, all on the
    problem's HIP stream; the owner -> slot tables are matched once, here."""

    def __init__(self, prob, win, info):
        self.prob = prob
        kf_owner, lm_owner = publish_owners(info)
        self.counts = prob.farm_plan(win.kf_gid, kf_owner, win.lm_gid, lm_owner)

    def exchange(self, prob=None):
        (prob or self.prob).farm_exchange()


class HostExchange:
    """The same exchange for stand-in problems on the CPU (state() / set_state() over numpy; gloo): the
    engine's buffer layout (per rank: published keyframes q t v, then landmarks), its matching
    (lba_farm_match, host-only C), one all_gather, vectorised pack / unpack."""

    KF = 13   # FARM_KF: q (4), t (3), velocity (6)

    def __init__(self, win, info, rank, world, group=None):
        import amc_lba
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank, self.world = rank, world
        kf_owner, lm_owner = publish_owners(info)
        self.pub_kf = np.nonzero(kf_owner == rank)[0]
        self.pub_lm = np.nonzero(lm_owner == rank)[0]
        cnt = self._gather(np.array([self.pub_kf.size, self.pub_lm.size], dtype=np.float64)).reshape(world, 2)
        self.kcap, self.lcap = int(cnt[:, 0].max()), int(cnt[:, 1].max())
        ids = np.full(self.kcap + self.lcap, -1.0)
        ids[: self.pub_kf.size] = win.kf_gid[self.pub_kf]
        ids[self.kcap: self.kcap + self.pub_lm.size] = win.lm_gid[self.pub_lm]
        ids = self._gather(ids).reshape(world, -1).astype(np.int64)
        sk, self.unmatched_kf = amc_lba.farm_match(rank, world, self.kcap, ids[:, : self.kcap], win.kf_gid, kf_owner)
        sl, self.unmatched_lm = amc_lba.farm_match(rank, world, self.lcap, ids[:, self.kcap:], win.lm_gid, lm_owner)
        self.stride = self.kcap * self.KF + 3 * self.lcap
        self.recv_kf = np.nonzero(sk >= 0)[0]
        o, i = np.divmod(sk[self.recv_kf], max(self.kcap, 1))
        self.src_kf = o * self.stride + i * self.KF
        self.recv_lm = np.nonzero(sl >= 0)[0]
        o, i = np.divmod(sl[self.recv_lm], max(self.lcap, 1))
        self.src_lm = o * self.stride + self.kcap * self.KF + 3 * i

    def _gather(self, a):
        t = self.torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return self.torch.cat(out).numpy()

    def exchange(self, prob):
        """prob: anything with state() -> (kfs, lm) and set_state(kfs=, lm=)."""
        kfs, lm = prob.state()
        mine = np.zeros(self.stride)
        kst = np.concatenate([kfs["q"], kfs["t"], kfs["vel"]], axis=1)   # the engine's state-record prefix
        mine[: self.pub_kf.size * self.KF] = kst[self.pub_kf].ravel()
        mine[self.kcap * self.KF: self.kcap * self.KF + 3 * self.pub_lm.size] = lm[self.pub_lm].ravel()
        buf = self._gather(mine)
        kfs_new, lm_new = kfs.copy(), lm.copy()
        rows = buf[self.src_kf[:, None] + np.arange(self.KF)[None, :]]
        kfs_new["q"][self.recv_kf] = rows[:, 0:4]
        kfs_new["t"][self.recv_kf] = rows[:, 4:7]
        kfs_new["vel"][self.recv_kf] = rows[:, 7:13]
        lm_new[self.recv_lm] = buf[self.src_lm[:, None] + np.arange(3)[None, :]]
        prob.set_state(kfs=kfs_new, lm=lm_new)
        return lm_new, kfs_new
