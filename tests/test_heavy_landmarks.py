"""Heavy landmarks: long tracks that one tile of k_lin_schur cannot hold.

LocalGPBA adds every observation of every local map point (src/Optimizer.cc:1050-1200): with bLarge up
to 25 optimisable keyframes plus covisible ones, and GP observations from non-keyframes, so a point can
be seen from more keyframes than a tile takes (TILE_KF = 16 pose blocks, 128 observations, 288 rows,
64 pose samples).  Such a landmark goes last in device order, is linearised in segment tiles, and its
segments are merged and eliminated by k_expand (heavy_item: g2o's Schur loop over every KF pair of the
landmark, block_solver.hpp:381-432).

CPU: the windows really contain heavy landmarks (counted on the host the way the device classifies
them).  GPU (through the C ABI, tolerances of tests/test_gpu_parity.py): residuals / H / b, damped steps
and whole LM runs against the oracle.
"""
from dataclasses import replace

import numpy as np
import pytest

import orc
from amc_lba.abi import MONO, MONO_GP
from amc_lba.synth import make_window

TILE_KF, TILE_OBS = 16, 128


def _consistent(win, extra, seed):
    """Append `extra` observations with measurements consistent with the window's estimate: the oracle's
    projection (the residual of z = 0, e = z - proj) plus one pixel of noise.  Only observations a
    tracker could have made are kept: depth test passed and the projection inside the 960 x 600 image
    (the generator's visibility rule)."""
    rng = np.random.default_rng(seed)
    extra = extra.copy()
    extra["z"] = 0.0
    w = replace(win, obs=np.concatenate([win.obs, extra]))
    o = orc.Oracle(w)
    _, res, _ = o.errors()
    ok = o.depth_ok().astype(bool)
    n0 = len(win.obs)
    z = -res[n0:]
    z[:, :2] += rng.normal(0, 1.0, (len(extra), 2))
    extra["z"] = z
    keep = ok[n0:] & (z[:, 0] >= 0) & (z[:, 0] < 960.0) & (z[:, 1] >= 0) & (z[:, 1] < 600.0)
    return replace(win, obs=np.concatenate([win.obs, extra[keep]]))


def _spanning(n_opt_kf=30, n_lm=300, n_long=5, seed=9, cams=(0, 3), repeat=1):
    """A window where n_long landmarks are also seen from every optimisable KF through the given cameras
    (the asynchronous cameras as GP observations between KF k - 1 and k, the reference camera 3 as a
    plain monocular one), each view `repeat` times (independent noise)."""
    win = make_window(n_opt_kf=n_opt_kf, n_lm=n_lm, obs_per_lm=6, n_cam=4, gp=True, seed=seed)
    kf_t = win.kfs["time"]
    rows = []
    for l in range(n_long):
        for k in range(2, len(win.kfs)):
            for c in [c for c in cams for _ in range(repeat)]:
                r = np.zeros(1, win.obs.dtype)
                r["lm"] = l
                r["kf_b"] = k
                r["cam"] = c
                r["w"] = 1.0
                if c == 3:
                    r["kind"], r["kf_a"], r["t"] = MONO, -1, kf_t[k]
                else:
                    r["kind"], r["kf_a"], r["t"] = MONO_GP, k - 1, kf_t[k] - 0.03
                rows.append(r)
    return _consistent(win, np.concatenate(rows), seed)


WINDOWS = {
    # 5 landmarks seen from ~30 KFs (GP observations couple KF k - 1 and k as well)
    "spanning": lambda: _spanning(),
    # > 128 observations per landmark (segments split on the observation limit too)
    "many_obs": lambda: _spanning(n_opt_kf=60, n_lm=400, n_long=3, seed=10, cams=(0, 1, 2, 3), repeat=3),
    # natural long tracks: geometric track lengths up to 60 over a 41-KF visibility band
    "long_tracks": lambda: make_window(n_opt_kf=50, n_lm=3000, obs_per_lm=8, track="geometric", max_track=60,
                                       band=41, seed=31),
}


def _heavy_count(win):
    """Landmarks the device path treats as heavy (more pose blocks or observations than a tile holds)."""
    o = win.obs
    fixed = win.kfs["fixed"].astype(bool)
    blocks = [set() for _ in range(len(win.lm))]
    for lm, kb, ka in zip(o["lm"], o["kf_b"], o["kf_a"]):
        for k in (kb, ka):
            if k >= 0 and not fixed[k]:
                blocks[lm].add(int(k))
    cnt = np.bincount(o["lm"], minlength=len(win.lm))
    return sum(1 for l in range(len(win.lm)) if len(blocks[l]) > TILE_KF or cnt[l] > TILE_OBS)


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("name", list(WINDOWS))
def test_windows_hold_heavy_landmarks(name):
    win = WINDOWS[name]()
    assert _heavy_count(win) >= 3
    if name == "many_obs":
        assert np.bincount(win.obs["lm"]).max() > TILE_OBS


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(WINDOWS))
def test_gpu_heavy_linearize_and_step_match_oracle(name):
    from amc_lba import Problem
    win = WINDOWS[name]()
    o = orc.Oracle(win)
    chi_o, res_o, c2_o = o.errors()
    H_o, b_o, Hll_o = o.build_system()
    p = Problem(win)
    res, H, b, Hll = p.linearize()
    assert np.linalg.norm(res - res_o) / np.linalg.norm(res_o) <= 1e-8
    assert _rel(H, H_o) < 1e-9 and _rel(b, b_o) < 1e-9 and _rel(Hll, Hll_o) < 1e-9
    chi, c2, _ = p.eval()
    assert abs(chi - chi_o) <= 1e-9 * chi_o
    for lam in (1.0, 1e-3):
        ok_o, dx_o = o.solve(lam)
        ok, dx = p.solve_step(lam)
        assert ok and ok_o
        n = p.pose_dim
        assert _rel(dx[:n], dx_o[:n]) <= 1e-6 and _rel(dx[n:], dx_o[n:]) <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(WINDOWS))
def test_gpu_heavy_optimize_matches_oracle(name):
    from amc_lba import Problem
    win = WINDOWS[name]()
    o = orc.Oracle(win)
    n_o, st_o = o.optimize(10)
    kf_o, lm_o = o.state()
    p = Problem(win)
    n, st = p.optimize(10)
    kf, lm = p.state()
    assert n == n_o and st.trials == st_o.trials and st.result == st_o.result
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6 and _rel(lm, lm_o) <= 1e-6
    # the last trial's per-observation chi2 (g2o's e->chi2() after optimize) and the depth flags
    np.testing.assert_allclose(p.trial_chi2(), o.last_obs_chi2(), rtol=1e-6, atol=1e-9)
    _, _, ok = p.eval()
    np.testing.assert_array_equal(ok, o.depth_ok())
