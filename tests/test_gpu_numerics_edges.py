"""GPU parity on the numerically exceptional paths of the reference, through the C ABI:

- the reduced camera system's factorisation failing (LinearSolverDense: `!isPositive()`,
  Thirdparty/g2o/g2o/solvers/linear_solver_dense.h:108-112): the damped step reports failure, and inside LM the
  trial's chi2 becomes DBL_MAX with BlockSolver's stale x applied (optimization_algorithm_levenberg.cpp:
  120-155), exactly as the oracle does;
- the small-angle branches the kernels take on the device: Sophus exp / log at epsilon = 1e-10
  (Thirdparty/Sophus/sophus/common.hpp:94), LeftJacobianPose3Q's series below |w| = 1e-5 and LeftJacobianRot3's
  identity below |w|^2 = DBL_EPSILON (src/Pose3utils.cc:11-21,50,63): evaluated on the GPU at the golden
  tangents (tests/golden, made from the reference's vendored Sophus sympy package), and exercised end to end by
  a window driving a straight line (zero relative rotations at the first linearisation).

Tolerances are the north-star's (residuals 1e-8, steps / states 1e-6) and the golden tests' own."""
import json
import os

import numpy as np
import pytest

import amc_lba
import orc
from amc_lba import Problem
from amc_lba.abi import FLAG_HOST_LOOP
from amc_lba.synth import make_window

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
GP_SMALL = dict(n_opt_kf=6, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=1)
# Qc with a negative z entry: EdgeVelocity's information QcInv(2,2) and the motion priors' QiInv(dt) are then
# indefinite, so H + lambda I is not positive for small lambda (the factorisation fails) and becomes positive
# once LM has raised lambda far enough (the trial succeeds)
QC_INDEFINITE = (0.02, 0.02, -20.0, 0.002, 0.002, 0.002)


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("lam", [-1e6, -1.0])
def test_solve_step_indefinite_fails_like_oracle(lam):
    """H + lambda I with lambda < 0 far below H's smallest eigenvalue: both factorisations report failure."""
    win = make_window(**GP_SMALL)
    o = orc.Oracle(win)
    o.build_system()
    ok_o, _ = o.solve(lam)
    p = Problem(win)
    p.linearize()
    ok, _ = p.solve_step(lam)
    assert not ok and not ok_o


def test_solve_step_indefinite_system_fails_then_recovers():
    win = make_window(**GP_SMALL)
    o = orc.Oracle(win, qc_diag=QC_INDEFINITE)
    o.build_system()
    p = Problem(win, qc_diag=QC_INDEFINITE)
    p.linearize()
    outcomes = []
    for lam in (1.0, 1e7):
        ok_o, dx_o = o.solve(lam)
        ok, dx = p.solve_step(lam)
        assert bool(ok) == bool(ok_o), lam
        outcomes.append(bool(ok))
        if ok:
            assert _rel(dx[:p.pose_dim], dx_o[:p.pose_dim]) <= 1e-6
    assert outcomes == [False, True]


@pytest.mark.parametrize("flags", [0, FLAG_HOST_LOOP])
def test_lm_with_failing_factorisations_matches_oracle(flags):
    """A whole LM run in which trials fail their factorisation (chi2 = DBL_MAX, lambda *= ni, the stale x)
    and later trials succeed: iterations, trials, solve failures, chi2 and the final states as the oracle,
    in the device-decided (queued) loop and the host-driven loop."""
    win = make_window(**GP_SMALL)
    o = orc.Oracle(win, qc_diag=QC_INDEFINITE, early_stop=0)
    n_o, st_o = o.optimize(10)
    kf_o, lm_o = o.state()
    assert st_o.solve_failures > 0 and st_o.trials > st_o.solve_failures + 1   # failures, and successes
    p = Problem(win, qc_diag=QC_INDEFINITE, early_stop=0, flags=flags)
    n, st = p.optimize(10)
    kf, lm = p.state()
    assert (n, st.trials, st.solve_failures, st.result) == (n_o, st_o.trials, st_o.solve_failures, st_o.result)
    assert abs(st.chi2_initial - st_o.chi2_initial) <= 1e-9 * abs(st_o.chi2_initial)
    assert st.chi2_final == st_o.chi2_final or abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * abs(st_o.chi2_final)
    assert abs(st.lambda_final - st_o.lambda_final) <= 1e-9 * abs(st_o.lambda_final)
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6
    assert _rel(kf["vel"], kf_o["vel"]) <= 1e-6
    assert _rel(lm, lm_o) <= 1e-6


def _golden_cases():
    se3 = json.load(open(os.path.join(GOLD, "sophus_golden.json")))["se3"]
    jac = json.load(open(os.path.join(GOLD, "se3_jacobian_golden.json")))["se3_right_jacobian"]
    return se3, jac


def test_device_exp_log_vs_sophus_golden():
    se3, _ = _golden_cases()
    xi = np.array([c["xi"] for c in se3])
    r = amc_lba.debug_lie(xi, q=np.array([c["q"] for c in se3]), t=np.array([c["t"] for c in se3]))
    for i, c in enumerate(se3):
        qg = np.array(c["q"])
        q = r["q"][i] * (1.0 if np.dot(r["q"][i], qg) >= 0 else -1.0)
        np.testing.assert_allclose(q, qg, atol=1e-13)
        np.testing.assert_allclose(r["t"][i], c["t"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(r["log"][i], c["log"], rtol=1e-10, atol=1e-10)


def test_device_right_jacobians_vs_golden():
    """Jr from the reference's sympy derivative of exp (80 digits), tolerances as the oracle's pin
    (tests/test_oracle_golden.py): exact branches 1e-13, the series branch 2e-11, the identity branch |w|."""
    _, jac = _golden_cases()
    xi = np.array([c["xi"] for c in jac])
    r = amc_lba.debug_lie(xi)
    for i, c in enumerate(jac):
        J = np.array(c["Jr"]).reshape(6, 6)
        th = np.linalg.norm(xi[i, 3:])
        tol = 1e-13 if th > 1e-4 else (2e-11 if th * th > np.finfo(float).eps else th)
        assert np.abs(r["Jr"][i] - J).max() <= tol * max(1.0, np.abs(J).max()), (xi[i], np.abs(r["Jr"][i] - J).max())
        assert np.abs(r["Jr_inv"][i] @ J - np.eye(6)).max() <= 10 * tol * max(1.0, np.abs(J).max()), xi[i]


def test_device_small_angle_branches_vs_oracle():
    """Tangents on both sides of every threshold (|w| = 0, 1e-12, 1e-10 +- (Sophus), 1e-8 = sqrt(eps) +-
    (LeftJacobianRot3), 1e-5 +- (LeftJacobianPose3Q), pi about x) against the oracle's restatement of the
    same branches."""
    base = np.array([0.4, -0.3, 0.2])
    dirs = np.array([1.0, -2.0, 0.5]) / np.linalg.norm([1.0, -2.0, 0.5])
    norms = [0.0, 1e-12, 0.99e-10, 1.01e-10, 1e-9, 1.4e-8, 1.5e-8, 0.99e-5, 1.01e-5, 1e-4, 0.3]
    xi = [np.concatenate([base, n * dirs]) for n in norms] + [np.array([0.3, -0.2, 0.1, np.pi, 0.0, 0.0]),
                                                           np.array([0.3, -0.2, 0.1, np.pi - 1e-9, 0.0, 0.0])]
    xi = np.array(xi)
    qs, ts = zip(*(orc.se3_exp(x) for x in xi))
    r = amc_lba.debug_lie(xi, q=np.array(qs), t=np.array(ts))
    for i, x in enumerate(xi):
        th = np.linalg.norm(x[3:])
        # between the thresholds the reference's closed forms cancel catastrophically ((th - sin th) / th^3 in
        # Sophus' V, 1 - sin(th) / th in LeftJacobianRot3, the LeftJacobianPose3Q coefficients): the kernels'
        # half-angle forms and the oracle's sin / cos forms agree to that cancellation (1e-10 .. 1e-12 on the
        # host build, tests/native/math_harness.cpp), not to rounding
        tol = 1e-9 if 1e-10 < th < 1e-3 else 1e-13
        q_o, t_o = orc.se3_exp(x)
        q = r["q"][i] * (1.0 if np.dot(r["q"][i], q_o) >= 0 else -1.0)
        np.testing.assert_allclose(q, q_o, atol=1e-15)
        np.testing.assert_allclose(r["t"][i], t_o, atol=tol)
        lg = orc.se3_log(np.array(qs[i]), np.array(ts[i]))
        if abs(np.linalg.norm(x[3:]) - np.pi) < 1e-6:   # log at pi: the rotation's sign is a free choice
            np.testing.assert_allclose(np.abs(r["log"][i][3:]), np.abs(lg[3:]), atol=1e-9)
        else:
            np.testing.assert_allclose(r["log"][i], lg, atol=1e-13)
        Jo, Jio = orc.right_jac_pose3(x), orc.right_jac_pose3_inv(x)
        assert np.abs(r["Jr"][i] - Jo).max() <= tol * max(1.0, np.abs(Jo).max()), (th, np.abs(r["Jr"][i] - Jo).max())
        assert np.abs(r["Jr_inv"][i] - Jio).max() <= tol * max(1.0, np.abs(Jio).max()), (th, np.abs(r["Jr_inv"][i] - Jio).max())


def test_straight_window_linearize_and_optimize_match_oracle():
    """A vehicle driving a straight line: every keyframe orientation and angular velocity equal, so the GP
    pairs' relative rotations, the samples' interpolated rotations and the velocities' omega are zero at the
    first linearisation (the series / identity branches of the kernels' Jacobians); LM then moves them off
    zero by the step.  Residuals, H, b, the step and the LM run against the oracle."""
    win = make_window(n_opt_kf=8, n_lm=400, obs_per_lm=6, n_cam=4, gp=True, seed=11, straight=True)
    q = win.kfs["q"]
    assert np.all(q == q[0]) and np.all(win.kfs["vel"][:, 3:] == 0.0)
    o = orc.Oracle(win)
    chi_o, res_o, _ = o.errors()
    H_o, b_o, _ = o.build_system()
    ok_o, dx_o = o.solve(1.0)
    p = Problem(win)
    res, H, b, _ = p.linearize()
    assert np.linalg.norm(res - res_o) / np.linalg.norm(res_o) <= 1e-8
    assert _rel(H, H_o) < 1e-9 and _rel(b, b_o) < 1e-9
    ok, dx = p.solve_step(1.0)
    assert ok and ok_o
    assert _rel(dx[:p.pose_dim], dx_o[:p.pose_dim]) <= 1e-6 and _rel(dx[p.pose_dim:], dx_o[p.pose_dim:]) <= 1e-6
    o2 = orc.Oracle(win)
    n_o, st_o = o2.optimize(10)
    kf_o, lm_o = o2.state()
    p2 = Problem(win)
    n, st = p2.optimize(10)
    kf, lm = p2.state()
    assert (n, st.trials, st.result) == (n_o, st_o.trials, st_o.result)
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6 and _rel(lm, lm_o) <= 1e-6
