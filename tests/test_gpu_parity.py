"""Parity of the HIP path (through the C ABI) against the CPU oracle on identical inputs.

Tolerances (BASELINE.json north_star): residual norm <= 1e-8 relative; pose update of one LM step
<= 1e-6 relative.  H/b blocks are held to 1e-9 relative to their maximum (summation order differs:
g2o adds edge by edge, the kernels reduce per tile segment).  Integer outputs (iterations, trial
counts, depth flags) must be identical.
"""
import ctypes
import os

import numpy as np
import pytest

import orc
from amc_lba import LbaError, Problem
from amc_lba.abi import LBA_E_EMPTY, LBA_E_LIMIT, MONO_GP, STEREO_GP, PRIOR_DTYPE
from amc_lba.synth import make_config_window, make_window

pytestmark = pytest.mark.gpu

WINDOWS = {
    "gp_small": dict(n_opt_kf=6, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=1),
    "gp_stereo": dict(n_opt_kf=5, n_lm=250, obs_per_lm=6, n_cam=3, gp=True, stereo_frac=1.0, seed=2),
    "mono_only": dict(n_opt_kf=9, n_fixed=1, n_lm=400, obs_per_lm=5, n_cam=1, gp=False, seed=3),
    "two_fixed": dict(n_opt_kf=6, n_fixed=2, n_lm=300, obs_per_lm=6, n_cam=4, gp=True, seed=4),
    "global_shape": dict(n_opt_kf=11, n_fixed=1, n_lm=500, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=5),
    # BundleAdjustment shape with 37 factorisation panels (deep dependent chain, banded S)
    "global_mid": dict(n_opt_kf=99, n_fixed=1, n_lm=8000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=6),
}


def _win(name):
    return make_window(**WINDOWS[name])


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("name", list(WINDOWS))
def test_linearize_matches_oracle(name):
    win = _win(name)
    o = orc.Oracle(win)
    chi_o, res_o, c2_o = o.errors()
    H_o, b_o, Hll_o = o.build_system()
    p = Problem(win)
    res, H, b, Hll = p.linearize()
    dres = np.linalg.norm(res - res_o) / np.linalg.norm(res_o)
    assert dres <= 1e-8, dres
    assert H.shape == H_o.shape
    assert _rel(H, H_o) < 1e-9
    assert _rel(b, b_o) < 1e-9
    assert _rel(Hll, Hll_o) < 1e-9
    chi, c2, _ = p.eval()
    assert abs(chi - chi_o) <= 1e-9 * chi_o
    np.testing.assert_allclose(c2, c2_o, rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("name", list(WINDOWS))
@pytest.mark.parametrize("lam", [1.0, 1e-3])
def test_solve_step_matches_oracle(name, lam):
    win = _win(name)
    o = orc.Oracle(win)
    o.build_system()
    ok_o, dx_o = o.solve(lam)
    p = Problem(win)
    p.linearize()
    ok, dx = p.solve_step(lam)
    assert ok == ok_o
    np_ = p.pose_dim
    assert _rel(dx[:np_], dx_o[:np_]) <= 1e-6
    assert _rel(dx[np_:], dx_o[np_:]) <= 1e-6


@pytest.mark.parametrize("name", list(WINDOWS))
def test_optimize_matches_oracle(name):
    win = _win(name)
    o = orc.Oracle(win)
    n_o, st_o = o.optimize(10)
    kf_o, lm_o = o.state()
    p = Problem(win)
    n, st = p.optimize(10)
    kf, lm = p.state()
    assert n == n_o
    assert st.trials == st_o.trials
    assert st.result == st_o.result
    assert abs(st.chi2_initial - st_o.chi2_initial) <= 1e-9 * st_o.chi2_initial
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6
    assert _rel(kf["vel"], kf_o["vel"]) <= 1e-5
    q, qo = kf["q"] * np.sign(kf["q"][:, 3:4]), kf_o["q"] * np.sign(kf_o["q"][:, 3:4])
    assert np.abs(q - qo).max() <= 1e-7
    assert _rel(lm, lm_o) <= 1e-6
    _, _, ok = p.eval()
    np.testing.assert_array_equal(ok, o.depth_ok())


def test_fixed_iteration_mode_runs_all_iterations():
    win = _win("gp_small")
    p = Problem(win, early_stop=0)
    n, st = p.optimize(15)
    assert n == 15 and st.iterations == 15
    o = orc.Oracle(win, early_stop=0)
    n_o, st_o = o.optimize(15)
    assert st.trials == st_o.trials
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final


def test_cfg1_full_size_linearize_and_step_parity():
    """BASELINE config 1 (50 KF / 20k landmarks / ~120k observations, 4 async cameras)."""
    win = make_config_window("cfg1_local_50kf")
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
    assert _rel(dx[:p.pose_dim], dx_o[:p.pose_dim]) <= 1e-6
    assert _rel(dx[p.pose_dim:], dx_o[p.pose_dim:]) <= 1e-6


def test_cfg1_full_size_optimize_matches_oracle():
    """BASELINE config 1 end to end: the reference's optimize(10) loop
    (Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-169, early stop disabled so
    all ten iterations run) on the GPU against the oracle: iterations, trials, chi2, keyframe
    poses / velocities and landmarks."""
    win = make_config_window("cfg1_local_50kf")
    o = orc.Oracle(win, early_stop=0)
    n_o, st_o = o.optimize(10)
    kf_o, lm_o = o.state()
    p = Problem(win, early_stop=0)
    n, st = p.optimize(10)
    kf, lm = p.state()
    assert n == n_o == 10
    assert st.trials == st_o.trials
    assert st.result == st_o.result
    assert abs(st.chi2_initial - st_o.chi2_initial) <= 1e-9 * st_o.chi2_initial
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6
    assert _rel(kf["vel"], kf_o["vel"]) <= 1e-6
    q, qo = kf["q"] * np.sign(kf["q"][:, 3:4]), kf_o["q"] * np.sign(kf_o["q"][:, 3:4])
    assert np.abs(q - qo).max() <= 1e-7
    assert _rel(lm, lm_o) <= 1e-6
    _, c2, ok = p.eval()
    np.testing.assert_array_equal(ok, o.depth_ok())


def test_cfg1_full_size_lm_properties():
    win = make_config_window("cfg1_local_50kf")
    p = Problem(win, early_stop=0)
    n, st = p.optimize(5)
    assert n == 5 and st.chi2_final < st.chi2_initial
    # deterministic: a second run from the same window is bitwise identical
    p2 = Problem(win, early_stop=0)
    n2, st2 = p2.optimize(5)
    assert st2.chi2_final == st.chi2_final and st2.trials == st.trials
    kf1, lm1 = p.state()
    kf2, lm2 = p2.state()
    assert np.array_equal(lm1, lm2) and np.array_equal(kf1["t"], kf2["t"])


def test_cfg2_global_full_size_parity():
    """BASELINE config 2 (global BA: 500 KF / 200k landmarks / 1.2M observations, S = 5988^2).
    Residuals, H_pp and b against the oracle at full size; the damped step through the
    size-independent normal-equation residual (H + lambda I) dx - b (the oracle's pivoted dense
    LDLT takes ~50 s at this size; global_mid checks dx itself); LM descent and determinism."""
    win = make_config_window("cfg2_global_500kf")
    o = orc.Oracle(win)
    chi_o, res_o, _ = o.errors()
    H_o, b_o, _ = o.build_system()
    p = Problem(win, early_stop=0)
    res, H, b, _ = p.linearize()
    assert np.linalg.norm(res - res_o) / np.linalg.norm(res_o) <= 1e-8
    assert _rel(H, H_o) < 1e-9 and _rel(b, b_o) < 1e-9
    del H, H_o
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


@pytest.mark.parametrize("early_stop", [1, 0])
def test_queued_loop_matches_host_loop(early_stop):
    """The device-decided (queued) LM loop takes exactly the decisions of the host-driven loop:
    same iterations / trials / results, bitwise-identical states and damping.  Long runs so rejected
    trials, multi-trial iterations and (early_stop=1) the TERMINATE exit all occur."""
    from amc_lba.abi import FLAG_HOST_LOOP
    rejected = 0
    cases = [(name, {}) for name in WINDOWS] + [("gp_small", dict(lambda_init=0.0)),
                                                 ("mono_only", dict(lambda_init=0.0, tau=1e-3))]
    for name, over in cases:   # lambda_init <= 0: computeLambdaInit (queued: on the device)
        win = _win(name)
        runs = []
        for flags in (0, FLAG_HOST_LOOP):
            p = Problem(win, early_stop=early_stop, flags=flags, **over)
            n, st = p.optimize(25)
            n2, st2 = p.optimize(3)   # a second call re-initialises lambda, like g2o
            kf, lm = p.state()
            runs.append((n, st, n2, st2, kf, lm))
        (n, st, n2, st2, kf, lm), (hn, hst, hn2, hst2, hkf, hlm) = runs
        assert (n, n2) == (hn, hn2), name
        for a, b in ((st, hst), (st2, hst2)):
            assert (a.iterations, a.trials, a.result, a.solve_failures) == \
                (b.iterations, b.trials, b.result, b.solve_failures), name
            assert a.chi2_initial == b.chi2_initial and a.chi2_final == b.chi2_final, name
            assert a.lambda_final == b.lambda_final, name
        assert np.array_equal(lm, hlm) and np.array_equal(kf["t"], hkf["t"]), name
        assert np.array_equal(kf["q"], hkf["q"]) and np.array_equal(kf["vel"], hkf["vel"]), name
        rejected += st.trials - st.iterations
    assert rejected > 0   # the multi-trial path was exercised


def test_stop_flag_stops_before_first_iteration():
    win = _win("gp_small")
    p = Problem(win)
    flag = ctypes.c_int32(1)
    n, st = p.optimize(10, stop_flag=flag)
    assert n == 0 and st.result == 2


def test_empty_graph_is_an_error():
    win = _win("gp_small")
    win.obs = win.obs[:0]
    win.priors = np.zeros(0, PRIOR_DTYPE)
    win.vel_kfs = win.vel_kfs[:0]
    p = Problem(win)
    with pytest.raises(LbaError) as ei:
        p.optimize(3)
    assert ei.value.code == LBA_E_EMPTY


def test_mfma_f64_layout(tmp_path):
    """The v_mfma_f64_16x16x4 lane layout k_lin_schur's Schur products rely on (exact integers)."""
    import subprocess
    src = os.path.join(os.path.dirname(__file__), "native", "mfma_f64_probe.hip")
    exe = str(tmp_path / "mfma_probe")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", src, "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_engine_reuse_across_windows_is_bitwise_fresh():
    """One engine, lba_set_problem with windows of different shapes one after another (the mapping thread's one
    problem per thread): each window's LM run equals a fresh engine's bitwise (no state of the
    previous window -- buffers, cached dissection plan, LM controller -- leaks into the next)."""
    names = ("gp_small", "global_mid", "mono_only", "gp_small")
    p = Problem(_win(names[0]))
    for i, name in enumerate(names):
        if i:
            p.set_window(_win(name))
        n, st = p.optimize(10)
        kfs, lm = p.state()
        q = Problem(_win(name))
        n2, st2 = q.optimize(10)
        kfs2, lm2 = q.state()
        q.close()
        assert (n, st.trials) == (n2, st2.trials), name
        assert st.chi2_final == st2.chi2_final, name
        assert kfs.tobytes() == kfs2.tobytes() and lm.tobytes() == lm2.tobytes(), name
    p.close()
