"""Extrinsic calibration (LocalGPBA bExtrinsic, src/Optimizer.cc:982-995, 1228-1240).

With lba_cam.ext_free the camera's VertexExtrinsic (include/G2oTypes.h:83-102) joins the pose system after
the keyframes (6 dofs each, g2o id order), linked by the camera's EdgeMonoGPExtrinsic observations
(_jacobianOplus[3], src/G2oTypes.cc:310-313) and an EdgeExtrinsicPrior (include/G2oTypes.h:470-494).

CPU (oracle): the extrinsic rows of b are -1/2 the central-difference gradient of the robust chi2 (those
Jacobians are exact); with every camera fixed the system is the one without extrinsics.
GPU (through the C ABI, tolerances of tests/test_gpu_parity.py): residuals / H / b, damped steps and whole
LM runs against the oracle, including the extrinsic estimates (lba_get_cams).
"""
from dataclasses import replace

import numpy as np
import pytest

import orc
from amc_lba.synth import make_window, with_free_extrinsics

SMALL = dict(n_opt_kf=6, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=11)


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def _ext_win(**over):
    kw = dict(SMALL)
    kw.update(over)
    return with_free_extrinsics(make_window(**kw))


def _perturb_cam(win, c, xi):
    """Tbc <- Tbc exp(xi) (VertexExtrinsic::oplusImpl)."""
    w = replace(win, cams=win.cams.copy())
    dq, dt = orc.se3_exp(np.asarray(xi, float))
    q1, t1 = w.cams[c]["q"] / np.linalg.norm(w.cams[c]["q"]), w.cams[c]["t"].copy()
    R1 = _qmat(q1)
    w.cams[c]["q"] = _qmul(q1, dq)
    w.cams[c]["t"] = R1 @ dt + t1
    return w


def _qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def test_oracle_extrinsic_gradient_matches_central_differences():
    win = _ext_win()
    o = orc.Oracle(win)
    n_kf_blocks = int((win.kfs["fixed"] == 0).sum())
    assert o.pose_dim == 12 * n_kf_blocks + 6 * 3
    o.errors()
    _, b, _ = o.build_system()
    h = 1e-6
    for c in range(3):
        for k in range(6):
            xi = np.zeros(6)
            xi[k] = h
            cp = orc.Oracle(_perturb_cam(win, c, xi)).errors()[0]
            cm = orc.Oracle(_perturb_cam(win, c, -xi)).errors()[0]
            g = (cp - cm) / (2 * h)
            bk = b[12 * n_kf_blocks + 6 * c + k]
            assert abs(-0.5 * g - bk) <= 2e-5 * max(abs(bk), 1.0), (c, k, -0.5 * g, bk)


def test_oracle_fixed_extrinsics_give_the_plain_system():
    win = make_window(**SMALL)
    o = orc.Oracle(win)
    o.errors()
    H0, b0, _ = o.build_system()
    w2 = _ext_win()
    w2.cams["ext_free"] = 0
    w2.cams["q"], w2.cams["t"] = win.cams["q"], win.cams["t"]
    o2 = orc.Oracle(w2)
    o2.errors()
    H1, b1, _ = o2.build_system()
    assert np.array_equal(H0, H1) and np.array_equal(b0, b1)


def test_oracle_calibration_moves_extrinsics_towards_truth():
    # (a 6-KF window leaves the extrinsics weakly observed; 30 KF / 3000 landmarks pin them)
    base = make_window(n_opt_kf=30, n_lm=3000, obs_per_lm=6, n_cam=4, gp=True, seed=12)
    win = with_free_extrinsics(base, rot_deg=0.5, trans=0.0)
    o = orc.Oracle(win, early_stop=0)
    n, st = o.optimize(10)
    assert st.chi2_final < st.chi2_initial
    cams = o.cams()
    for c in range(3):
        def ang(q):
            d = _qmul(np.array([-base.cams[c]["q"][0], -base.cams[c]["q"][1], -base.cams[c]["q"][2],
                                base.cams[c]["q"][3]]), q / np.linalg.norm(q))
            return 2 * np.arcsin(min(1.0, np.linalg.norm(d[:3])))
        assert ang(cams[c]["q"]) < ang(win.cams[c]["q"]), c


# ---------------------------------------------------------------------------------------------- GPU
EXT_WINDOWS = {
    "ext_small": dict(SMALL),
    "ext_mid": dict(n_opt_kf=30, n_lm=3000, obs_per_lm=6, n_cam=4, gp=True, seed=12),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(EXT_WINDOWS))
def test_gpu_extrinsic_linearize_and_step_match_oracle(name):
    from amc_lba import Problem
    win = _ext_win(**EXT_WINDOWS[name])
    o = orc.Oracle(win)
    chi_o, res_o, _ = o.errors()
    H_o, b_o, Hll_o = o.build_system()
    p = Problem(win)
    assert p.pose_dim == o.pose_dim
    res, H, b, Hll = p.linearize()
    assert np.linalg.norm(res - res_o) / np.linalg.norm(res_o) <= 1e-8
    assert _rel(H, H_o) < 1e-9 and _rel(b, b_o) < 1e-9 and _rel(Hll, Hll_o) < 1e-9
    chi, _, _ = p.eval()
    assert abs(chi - chi_o) <= 1e-9 * chi_o
    for lam in (1.0, 1e-3):
        ok_o, dx_o = o.solve(lam)
        ok, dx = p.solve_step(lam)
        assert ok and ok_o
        n = p.pose_dim
        assert _rel(dx[:n], dx_o[:n]) <= 1e-6 and _rel(dx[n:], dx_o[n:]) <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(EXT_WINDOWS))
def test_gpu_extrinsic_optimize_matches_oracle(name):
    from amc_lba import Problem
    win = _ext_win(**EXT_WINDOWS[name])
    o = orc.Oracle(win)
    n_o, st_o = o.optimize(10)
    kf_o, lm_o = o.state()
    cam_o = o.cams()
    p = Problem(win)
    n, st = p.optimize(10)
    kf, lm = p.state()
    cam = p.cams()
    assert n == n_o and st.trials == st_o.trials and st.result == st_o.result
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6 and _rel(lm, lm_o) <= 1e-6
    q, qo = cam["q"] * np.sign(cam["q"][:, 3:4]), cam_o["q"] * np.sign(cam_o["q"][:, 3:4])
    assert np.abs(q - qo).max() <= 1e-7
    assert _rel(cam["t"], cam_o["t"]) <= 1e-6
    assert np.array_equal(cam["q"][3], win.cams["q"][3])   # the reference camera stays fixed
    _, _, ok = p.eval()
    np.testing.assert_array_equal(ok, o.depth_ok())


@pytest.mark.gpu
def test_gpu_extrinsic_argument_errors():
    """EdgeStereoGP projects through the static MultiKeyFrame::mTbc, so a stereo GP observation of a camera
    with a free extrinsic is rejected (LBA_E_ARG); a partitioned problem does not take free extrinsics
    (LBA_E_LIMIT)."""
    from amc_lba import Group, LbaError, Problem
    from amc_lba.abi import LBA_E_ARG, LBA_E_LIMIT, STEREO_GP
    win = _ext_win(stereo_frac=0.0)
    bad = replace(win, obs=win.obs.copy())
    i = int(np.nonzero(bad.obs["kind"] == 0)[0][0])
    bad.obs["kind"][i] = STEREO_GP
    with pytest.raises(LbaError) as ei:
        Problem(bad)
    assert ei.value.code == LBA_E_ARG
    # (a single rank is not partitioned).  A failing rank releases its peers through the set-up status
    # all-reduce, so both ranks of the group call in (one alone would wait for its peer)
    import threading
    g = Group(2)
    codes = [None, None]

    def rank(r):
        try:
            Problem(win, group=g, rank=r)
        except LbaError as e:
            codes[r] = e.code
    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert codes == [LBA_E_LIMIT, LBA_E_LIMIT]
    g.close()
