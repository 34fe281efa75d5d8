"""Window farm exchange (BASELINE config 3) on CPU with the gloo backend, world_size 2.

Each rank holds a stand-in problem (state()/set_state() over numpy arrays — no GPU, no oracle);
after one window-boundary exchange every non-owned shared landmark / keyframe must equal the
owner's estimate, and owned vertices must be untouched."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from amc_lba import farm


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeProblem:
    def __init__(self, win, rank):
        self.kfs = win.kfs.copy()
        self.lm = win.lm.copy() + 1000.0 * rank      # make every rank's copy distinguishable
        self.kfs["t"] += 1000.0 * rank

    def state(self):
        return self.kfs.copy(), self.lm.copy()

    def set_state(self, kfs=None, lm=None):
        if kfs is not None:
            self.kfs = kfs.copy()
        if lm is not None:
            self.lm = lm.copy()


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wins, infos = farm.make_farm_windows("cfg1_local_50kf", world, seed=3, stride=25)
    win, info = wins[rank], infos[rank]
    prob = _FakeProblem(win, rank)
    ex = farm.HostExchange(win, info, rank, world)
    before_lm, before_kf = prob.lm.copy(), prob.kfs["t"].copy()
    ex.exchange(prob)
    q.put((rank, win.lm_gid, win.kf_gid, info.lm_owner, info.kf_owner, before_lm, before_kf, prob.lm, prob.kfs["t"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_shared_state_exchange_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, *rest = q.get(timeout=300)
        res[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0, k0, lo0, ko0, blm0, bkf0, lm0, kf0 = res[0]
    g1, k1, lo1, ko1, blm1, bkf1, lm1, kf1 = res[1]
    shared = np.intersect1d(g0, g1)
    assert shared.size > 1000                        # ~50 % overlap between neighbouring windows
    i0 = np.searchsorted(g0, shared)
    i1 = np.searchsorted(g1, shared)
    assert (lo0[i0] == 0).all() and (lo1[i1] == 0).all()
    np.testing.assert_array_equal(lm0[i0], blm0[i0])   # owner untouched
    np.testing.assert_array_equal(lm1[i1], blm0[i0])   # rank 1 received rank 0's estimate
    own1 = lo1 == 1
    np.testing.assert_array_equal(lm1[own1], blm1[own1])
    ks = np.intersect1d(k0, k1)
    assert ks.size == 26
    np.testing.assert_array_equal(kf1[np.searchsorted(k1, ks)], bkf0[np.searchsorted(k0, ks)])
