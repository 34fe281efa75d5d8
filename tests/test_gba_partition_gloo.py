"""Partitioned global BA (BASELINE config 4) on CPU with the gloo backend, world_size 2: the sum of
the ranks' pose systems (oracle, test infrastructure) equals the unpartitioned system, and every
rank's landmark blocks are the unpartitioned ones — the decomposition the GPU ranks all-reduce every
LM trial (amc_lba/gba.py, lba_set_partition)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

WIN = dict(n_opt_kf=30, n_fixed=1, n_lm=3000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "amc-slam_amd"), os.path.join(root, "oracle")]
    import torch.distributed as dist
    import orc
    from amc_lba.gba import partition_window
    from amc_lba.synth import make_window
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    win = make_window(**WIN)
    part, ids = partition_window(win, rank, world)
    o = orc.Oracle(part)
    chi, _, _ = o.errors()
    H, b, Hll = o.build_system()
    npose = H.shape[0]
    t = torch.from_numpy(np.concatenate([H.ravel(), b[:npose], [chi]]))
    dist.all_reduce(t)
    q.put((rank, t.numpy(), ids, b[npose:], Hll))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_partition_sums_to_full_system_world2():
    import orc
    from amc_lba.synth import make_window
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
    win = make_window(**WIN)
    o = orc.Oracle(win)
    chi, _, _ = o.errors()
    H, b, Hll = o.build_system()
    n = H.shape[0]
    summed = res[0][0]
    np.testing.assert_array_equal(summed, res[1][0])          # both ranks hold the same sums
    np.testing.assert_allclose(summed[: n * n].reshape(n, n), H, rtol=1e-12, atol=1e-9 * np.abs(H).max())
    np.testing.assert_allclose(summed[n * n: n * n + n], b[:n], rtol=1e-12, atol=1e-9 * np.abs(b[:n]).max())
    assert abs(summed[-1] - chi) <= 1e-12 * chi
    bl = b[n:].reshape(-1, 3)
    for r in range(world):
        _, ids, bl_r, Hll_r = res[r]
        np.testing.assert_allclose(bl_r.reshape(-1, 3), bl[ids], rtol=1e-12, atol=1e-12 * np.abs(bl).max())
        np.testing.assert_allclose(Hll_r, Hll[ids], rtol=1e-12)


# ---- the split of the distributed factorisation (LBA_FLAG_SUBTREE_SOLVE): lba_partition_assign on every rank
def _split_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "amc-slam_amd"), os.path.join(root, "oracle")]
    import torch.distributed as dist
    import amc_lba
    import orc
    from amc_lba.gba import partition_window
    from amc_lba.synth import make_window
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    win = make_window(**SPLIT_WIN)
    lm_r, pri_r, vel_r, panels, kf_r = amc_lba.partition_assign(win, world, kf=True)   # each rank on its own
    sig = torch.tensor([float(np.sum(lm_r * np.arange(1, len(lm_r) + 1) % 1000003)), float(np.sum(kf_r + 1)),
                        float(np.sum(pri_r)), float(panels[1])], dtype=torch.float64)
    sigs = [torch.zeros_like(sig) for _ in range(world)]
    dist.all_gather(sigs, sig)
    part, ids = partition_window(win, rank, world, (lm_r, pri_r, vel_r))
    # locality: every keyframe of the rank's edges is in its subtree or the top
    o_kf = np.concatenate([part.obs["kf_b"], part.obs["kf_a"][np.isin(part.obs["kind"], (0, 1))],
                           part.priors["kf_a"], part.priors["kf_b"], np.asarray(part.vel_kfs)])
    stray = int(np.sum((kf_r[o_kf] >= 0) & (kf_r[o_kf] != rank)))
    # the parts' chi2 (oracle) sums to the window's: every observation and edge on exactly one rank
    chi, _, _ = orc.Oracle(part).errors()
    t = torch.tensor([chi, float(len(part.obs)), float(len(part.priors))], dtype=torch.float64)
    dist.all_reduce(t)
    q.put((rank, [s.numpy() for s in sigs], stray, t.numpy(), len(ids), kf_r))
    dist.barrier()
    dist.destroy_process_group()


SPLIT_WIN = dict(n_opt_kf=59, n_fixed=1, n_lm=3000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=9)


@pytest.mark.slow
def test_subtree_split_layout_world2():
    """Both ranks derive the same split on their own; each rank's landmarks and edges only touch keyframes of
    its own subtree or of the top (so its subtree tiles of the reduced system are complete without any
    exchange: only the top is all-reduced); every observation and edge lands on exactly one rank."""
    import orc
    from amc_lba.synth import make_window
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, *rest = q.get(timeout=300)
        res[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sigs0 = res[0][0]
    np.testing.assert_array_equal(sigs0[0], sigs0[1])   # the same split on both ranks
    kf_r = res[0][4]
    assert (kf_r == 0).any() and (kf_r == 1).any() and (kf_r == -1).any()   # two subtrees and a top
    for r in range(world):
        assert res[r][1] == 0, f"rank {r} holds edges of the other rank's subtree"
    assert res[0][3] + res[1][3] == SPLIT_WIN["n_lm"]
    win = make_window(**SPLIT_WIN)
    chi, _, _ = orc.Oracle(win).errors()
    summed = res[0][2]
    assert summed[1] == len(win.obs) and summed[2] == len(win.priors)
    assert abs(summed[0] - chi) <= 1e-12 * chi


def test_partition_rejects_free_extrinsics():
    """A partitioned problem takes no free extrinsic (a partitioned lba_set_problem returns LBA_E_LIMIT before it plans,
    and lba_partition_assign plans the keyframe-only pattern): both Python entry points of the split refuse such a
    window up front, with the reason, instead of a rank failing later with a stray-landmark error."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "amc-slam_amd")]
    import amc_lba
    from amc_lba.abi import LBA_E_LIMIT
    from amc_lba.gba import partition_window
    from amc_lba.synth import make_window, with_free_extrinsics
    win = with_free_extrinsics(make_window(n_opt_kf=8, n_lm=400, obs_per_lm=6, n_cam=4, gp=True, stereo_frac=0.0,
                                           seed=3))
    with pytest.raises(amc_lba.LbaError) as ei:
        amc_lba.partition_assign(win, 2)
    assert ei.value.code == LBA_E_LIMIT and "extrinsic" in str(ei.value)
    with pytest.raises(ValueError, match="extrinsic"):
        partition_window(win, 0, 2)
    assert partition_window(win, 0, 1)[0] is win   # (one rank: not partitioned)
