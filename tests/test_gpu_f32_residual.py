"""The fp32-residual option (LBA_FLAG_F32_RESIDUAL; BASELINE.json configs[4]: "fp32 residuals + fp64 accumulate")
on the GPU, through the C ABI, against the fp64 oracle.

Each observation's projection, residual and Jacobian rows run in fp32 (k_lin_schur / k_update / k_eval's <true>
instantiations; the world offset Xw - twb stays fp64), every sum (J^T W J, J^T W e, the Schur complement, the
solve, chi2) in fp64.  Residuals carry fp32 rounding of pixel-scale values (<= ~1e-4 px, host check in
tests/test_math_host.py), so the tolerances are stated looser than the fp64 path's 1e-8 / 1e-9 and each test
also checks that the deviation is above fp64 rounding (the fp32 kernels really ran):
  residual vector     <= 1e-3 relative (norm)      chi2        <= 1e-4 relative
  H_pp, b             <= 1e-5 / 1e-4 of max        damped step <= 1e-3 relative (normal-equation residual at
                                                                   config 2: <= 1e-4 of max |b|)
  LM optimize(10)     final chi2 <= 1e-3 relative, keyframe positions / landmarks <= 1e-3 relative.
The fp64 default (tests/test_gpu_parity.py) is unchanged by the option: its kernels are the <false> instantiations.
"""
import numpy as np
import pytest

import orc
from amc_lba import Problem
from amc_lba.abi import FLAG_F32_RESIDUAL
from amc_lba.synth import make_config_window, make_window

pytestmark = pytest.mark.gpu

WINDOWS = {
    "gp_small": dict(n_opt_kf=6, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=1),
    "gp_stereo": dict(n_opt_kf=5, n_lm=250, obs_per_lm=6, n_cam=3, gp=True, stereo_frac=1.0, seed=2),
    "mono_only": dict(n_opt_kf=9, n_fixed=1, n_lm=400, obs_per_lm=5, n_cam=1, gp=False, seed=3),
    "global_mid": dict(n_opt_kf=99, n_fixed=1, n_lm=8000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=6),
}


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("name", list(WINDOWS))
def test_f32_residual_linearize_and_step_within_tolerance(name):
    win = make_window(**WINDOWS[name])
    o = orc.Oracle(win)
    chi_o, res_o, _ = o.errors()
    H_o, b_o, _ = o.build_system()
    ok_o, dx_o = o.solve(1.0)
    p = Problem(win, flags=FLAG_F32_RESIDUAL)
    res, H, b, _ = p.linearize()
    dres = np.linalg.norm(res - res_o) / np.linalg.norm(res_o)
    dH, db = _rel(H, H_o), _rel(b, b_o)
    chi, _, _ = p.eval()
    dchi = abs(chi - chi_o) / chi_o
    ok, dx = p.solve_step(1.0)
    ddx = _rel(dx, dx_o)
    p.close()
    print(f"{name}: residual {dres:.2e}  H {dH:.2e}  b {db:.2e}  chi2 {dchi:.2e}  dx {ddx:.2e}")
    assert 1e-9 < dres <= 1e-3, dres   # (above fp64 rounding: the fp32 kernels ran)
    assert dH <= 1e-5 and db <= 1e-4, (dH, db)
    assert dchi <= 1e-4, dchi
    assert ok and ok_o
    assert ddx <= 1e-3, ddx


@pytest.mark.parametrize("name", ["gp_small", "mono_only", "global_mid"])
def test_f32_residual_optimize_within_tolerance(name):
    win = make_window(**WINDOWS[name])
    o = orc.Oracle(win, early_stop=0)
    n_o, st_o = o.optimize(10)
    kf_o, lm_o = o.state()
    p = Problem(win, early_stop=0, flags=FLAG_F32_RESIDUAL)
    n, st = p.optimize(10)
    kf, lm = p.state()
    p.close()
    dchi = abs(st.chi2_final - st_o.chi2_final) / st_o.chi2_final
    dt, dl = _rel(kf["t"], kf_o["t"]), _rel(lm, lm_o)
    print(f"{name}: trials {st.trials} / {st_o.trials}  chi2 {dchi:.2e}  kf t {dt:.2e}  lm {dl:.2e}")
    assert n == n_o == 10
    assert st.chi2_final < st.chi2_initial
    assert dchi <= 1e-3, dchi
    assert dt <= 1e-3 and dl <= 1e-3, (dt, dl)
    # deterministic: a second run gives bitwise the same result
    p2 = Problem(win, early_stop=0, flags=FLAG_F32_RESIDUAL)
    n2, st2 = p2.optimize(10)
    kf2, lm2 = p2.state()
    p2.close()
    assert st2.chi2_final == st.chi2_final and st2.trials == st.trials
    assert np.array_equal(kf2["t"], kf["t"]) and np.array_equal(lm2, lm)


def test_f32_residual_cfg2_full_size():
    """BASELINE config 2 (global BA, 500 KF / 200k landmarks / 1.2M observations) with the option: residuals, H_pp
    and b against the fp64 oracle, the damped step through the normal-equation residual of the oracle's fp64
    system, and LM descent."""
    win = make_config_window("cfg2_global_500kf")
    o = orc.Oracle(win)
    chi_o, res_o, _ = o.errors()
    H_o, b_o, _ = o.build_system()
    p = Problem(win, early_stop=0, flags=FLAG_F32_RESIDUAL)
    res, H, b, _ = p.linearize()
    dres = np.linalg.norm(res - res_o) / np.linalg.norm(res_o)
    dH, db = _rel(H, H_o), _rel(b, b_o)
    del H, H_o
    lam = win.cfg["lambda_init"]
    ok, dx = p.solve_step(lam)
    r = o.normal_residual(lam, dx)
    dr = np.abs(r).max() / np.abs(b_o).max()
    n, st = p.optimize(3)
    p.close()
    print(f"cfg2: residual {dres:.2e}  H {dH:.2e}  b {db:.2e}  normal residual {dr:.2e}  "
          f"chi2 {st.chi2_initial:.6e} -> {st.chi2_final:.6e} (oracle chi2_0 {chi_o:.6e})")
    assert 1e-9 < dres <= 1e-3, dres
    assert dH <= 1e-5 and db <= 1e-4, (dH, db)
    assert ok and dr <= 1e-4, dr
    assert n == 3 and st.chi2_final < st.chi2_initial
    assert abs(st.chi2_initial - chi_o) <= 1e-4 * chi_o
