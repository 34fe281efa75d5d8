"""Band solve of the reduced camera system (k_chol_flow task kinds 4 / 5): after the dataflow
factorisation, forward and back substitution tasks over the envelope instead of the tiles of L^-1.
It is the path for pose systems above 6144 (global BA beyond 512 keyframes; the
reference solves those with LinearSolverEigen's SimplicialLDLT, linear_solver_eigen.h:50-233) and
can be forced on any window with LBA_FLAG_BAND_SOLVE.  Checked against the oracle's pivoted LDLT on
the small windows, against the L^-1 solve on config 2, and through the size-independent normal
equation residual (H + lambda I) dx - b above 6144."""
import numpy as np
import pytest

import orc
from amc_lba import LbaError, Problem
from amc_lba.abi import FLAG_BAND_SOLVE, FLAG_DENSE_SOLVE, LBA_E_LIMIT
from amc_lba.synth import make_config_window, make_window

pytestmark = pytest.mark.gpu

WINDOWS = {
    "gp_small": dict(n_opt_kf=6, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=1),
    "gp_stereo": dict(n_opt_kf=5, n_lm=250, obs_per_lm=6, n_cam=3, gp=True, stereo_frac=1.0, seed=2),
    "mono_only": dict(n_opt_kf=9, n_fixed=1, n_lm=400, obs_per_lm=5, n_cam=1, gp=False, seed=3),
    "global_shape": dict(n_opt_kf=11, n_fixed=1, n_lm=500, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=5),
    "global_mid": dict(n_opt_kf=99, n_fixed=1, n_lm=8000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=6),
}


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("name", list(WINDOWS))
def test_band_step_matches_oracle_and_dense(name):
    win = make_window(**WINDOWS[name])
    o = orc.Oracle(win)
    o.build_system()
    lam = 1.0
    ok_o, dx_o = o.solve(lam)
    pb = Problem(win, flags=FLAG_BAND_SOLVE)
    pb.linearize()
    ok, dx = pb.solve_step(lam)
    assert ok == ok_o
    n = pb.pose_dim
    assert _rel(dx[:n], dx_o[:n]) <= 1e-6 and _rel(dx[n:], dx_o[n:]) <= 1e-6
    pd = Problem(win, flags=FLAG_DENSE_SOLVE)
    pd.linearize()
    okd, dxd = pd.solve_step(lam)
    assert okd == ok
    assert _rel(dx, dxd) <= 1e-9   # same factorisation, different triangular-solve summation order


@pytest.mark.parametrize("name", list(WINDOWS))
def test_band_optimize_matches_oracle(name):
    win = make_window(**WINDOWS[name])
    o = orc.Oracle(win)
    n_o, st_o = o.optimize(10)
    kf_o, lm_o = o.state()
    p = Problem(win, flags=FLAG_BAND_SOLVE)
    n, st = p.optimize(10)
    kf, lm = p.state()
    assert n == n_o and st.trials == st_o.trials and st.result == st_o.result
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6 and _rel(lm, lm_o) <= 1e-6


def test_cfg2_band_matches_dense_solve():
    """BASELINE config 2 (S = 5988^2): the band solve and the L^-1 solve give the same step."""
    win = make_config_window("cfg2_global_500kf")
    lam = win.cfg["lambda_init"]
    steps = []
    for flags in (FLAG_BAND_SOLVE, FLAG_DENSE_SOLVE):
        p = Problem(win, flags=flags)
        p.linearize()
        ok, dx = p.solve_step(lam)
        assert ok
        steps.append(dx)
    assert _rel(steps[0], steps[1]) <= 1e-8


def test_large_pose_system_band_solve():
    """700 optimisable keyframes (pose system 8400 > 6144): the band path is taken automatically;
    the step satisfies the normal equations of the oracle's system, LM descends and is
    deterministic.  The L^-1 solve refuses this size."""
    win = make_window(n_opt_kf=700, n_fixed=1, n_lm=60000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True,
                      seed=12, name="global_700")
    with pytest.raises(LbaError) as ei:
        Problem(win, flags=FLAG_DENSE_SOLVE)
    assert ei.value.code == LBA_E_LIMIT
    o = orc.Oracle(win)
    chi_o, res_o, _ = o.errors()
    _, b_o, _ = o.build_system()
    p = Problem(win, early_stop=0)
    assert p.pose_dim == 8400
    res, _, b, _ = p.linearize()
    assert np.linalg.norm(res - res_o) / np.linalg.norm(res_o) <= 1e-8
    assert _rel(b, b_o) < 1e-9
    lam = win.cfg["lambda_init"]
    ok, dx = p.solve_step(lam)
    assert ok
    r = o.normal_residual(lam, dx)
    assert np.abs(r).max() <= 1e-8 * np.abs(b_o).max(), np.abs(r).max() / np.abs(b_o).max()
    n, st = p.optimize(3)
    assert n == 3 and st.chi2_final < st.chi2_initial
    assert abs(st.chi2_initial - chi_o) <= 1e-9 * chi_o
    p2 = Problem(win, early_stop=0)
    n2, st2 = p2.optimize(3)
    assert st2.chi2_final == st.chi2_final and st2.trials == st.trials


def test_pose_system_beyond_131040():
    """11 000 optimisable keyframes (pose system 132 000, 4125 panels: beyond the 12-bit panel codes of
    round 2): set up, solved through the band path with packed envelope storage, LM descent and
    bitwise determinism (the oracle's dense system would take 139 GB)."""
    win = make_window(n_opt_kf=11000, n_fixed=1, n_lm=44000, obs_per_lm=4, n_cam=1, gp=False, stereo_frac=0.0,
                      seed=11, global_ba=True, name="chain_11k")
    p = Problem(win, early_stop=0)
    assert p.pose_dim == 132000
    info = p.solver_info()
    assert info["panels"] > 4095 and info["band"] == 1
    assert p.device_bytes() < 4e9, p.device_bytes()
    n, st = p.optimize(2)
    assert n == 2 and st.chi2_final < st.chi2_initial
    kf, lm = p.state()
    p.close()
    p2 = Problem(win, early_stop=0)
    n2, st2 = p2.optimize(2)
    kf2, lm2 = p2.state()
    assert st2.chi2_final == st.chi2_final and st2.trials == st.trials
    np.testing.assert_array_equal(kf2["t"], kf["t"])
    np.testing.assert_array_equal(lm2, lm)
