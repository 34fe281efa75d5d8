"""Reduced camera systems of loop-closure shape: global BA over a
trajectory that comes back to its start, so S has long-range blocks between the first and the last
keyframes (the structure LoopClosing::RunGlobalBundleAdjustment hands to BundleAdjustment's
LinearSolverEigen, src/LoopClosing.cc:1206-1221, src/Optimizer.cc:70; linear_solver_eigen.h:94-124).
The rows of the last keyframes reach back to the first panel, which defeats the one-level dissection
[A | S1 | B] of the factorisation (the whole system becomes one dependent chain); the engine therefore
cuts off a tail separator S2 of such rows: [A | S1 | B | S2], factored as [A | B | S1 | S2], so A and B
stay concurrent (lba_solver_info: tail, chain).  Checked against the oracle's pivoted LDLT of the
whole system on the L^-1-tile and the substitution (band) solves, and against the dissection without a
tail (LBA_ND_NO_TAIL) on the same window.  A trajectory of three laps (every place revisited twice:
every lap couples every other one) needs the graph dissection (lba_plan.hpp); its chain, levels and
fill are reported by lba_solver_info."""
import os

import numpy as np
import pytest

import orc
from amc_lba import Problem
from amc_lba.abi import FLAG_BAND_SOLVE
from amc_lba.synth import make_config_window, make_window

pytestmark = pytest.mark.gpu

LAPS3 = dict(n_opt_kf=149, n_fixed=1, n_lm=12000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=7, loop=3)
LOOP_MID = dict(n_opt_kf=99, n_fixed=1, n_lm=8000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=6, loop=True)


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def _with_env(key, val, fn):
    os.environ[key] = val
    try:
        return fn()
    finally:
        del os.environ[key]


def _no_tail(fn):
    os.environ["LBA_ND_NO_TAIL"] = "1"
    try:
        return fn()
    finally:
        del os.environ["LBA_ND_NO_TAIL"]


def test_loop_window_has_long_range_blocks():
    win = make_window(**LOOP_MID)
    o = win.obs
    first = np.full(len(win.lm), 10 ** 9)
    last = np.zeros(len(win.lm), int)
    np.minimum.at(first, o["lm"], o["kf_b"])
    np.maximum.at(last, o["lm"], o["kf_b"])
    assert ((first < 10) & (last >= 90)).sum() > 100


@pytest.mark.parametrize("flags", [0, FLAG_BAND_SOLVE])
def test_loop_step_and_lm_match_oracle(flags):
    win = make_window(**LOOP_MID)
    o = orc.Oracle(win)
    chi_o, res_o, _ = o.errors()
    H_o, b_o, _ = o.build_system()
    lam = win.cfg["lambda_init"]
    ok_o, dx_o = o.solve(lam)
    p = Problem(win, flags=flags)
    info = p.solver_info()
    assert info["chain"] < 0.75 * info["panels"]
    assert info["band"] == int(flags == FLAG_BAND_SOLVE)
    res, H, b, _ = p.linearize()
    assert np.linalg.norm(res - res_o) / np.linalg.norm(res_o) <= 1e-8
    assert _rel(H, H_o) < 1e-9 and _rel(b, b_o) < 1e-9
    ok, dx = p.solve_step(lam)
    assert ok and ok_o
    n = p.pose_dim
    assert _rel(dx[:n], dx_o[:n]) <= 1e-6 and _rel(dx[n:], dx_o[n:]) <= 1e-6
    r = o.normal_residual(lam, dx)
    assert np.abs(r).max() <= 1e-8 * np.abs(b_o).max()
    o2 = orc.Oracle(win, early_stop=0)
    n_o, st_o = o2.optimize(6)
    p2 = Problem(win, early_stop=0, flags=flags)
    n2, st = p2.optimize(6)
    assert n2 == n_o and st.trials == st_o.trials
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final
    kf, lm = p2.state()
    kf_o, lm_o = o2.state()
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6 and _rel(lm, lm_o) <= 1e-6


def test_loop_tail_shortens_the_chain_same_step():
    """The interval dissection (LBA_ND_METHOD=1) needs the loop-closure tail; the graph dissection (the
    default picks the shorter chain of the two) needs none.  All give the same step."""
    win = make_window(**LOOP_MID)
    lam = win.cfg["lambda_init"]

    def run():
        p = Problem(win, flags=FLAG_BAND_SOLVE)
        p.linearize()
        ok, dx = p.solve_step(lam)
        assert ok
        return p.solver_info(), dx

    without = _with_env("LBA_ND_METHOD", "1", lambda: _no_tail(run))
    with_tail = _with_env("LBA_ND_METHOD", "1", run)
    graph = _with_env("LBA_ND_METHOD", "2", run)
    best = run()
    assert without[0]["tail"] == 0 and with_tail[0]["tail"] > 0 and graph[0]["tail"] == 0
    assert with_tail[0]["chain"] < 0.75 * without[0]["chain"]
    assert best[0]["chain"] == min(with_tail[0]["chain"], graph[0]["chain"])
    for other in (without, with_tail, graph):
        assert _rel(other[1], best[1]) <= 1e-8


def test_dissection_depth_cap_same_step():
    """LBA_ND_LEVELS caps the nested dissection's depth (0: the natural panel order, one dependent chain): the same
    step on the config-1 window as the default plan, through a longer chain."""
    win = make_config_window("cfg1_local_50kf")
    lam = win.cfg["lambda_init"]

    def run():
        p = Problem(win)
        p.linearize()
        ok, dx = p.solve_step(lam)
        assert ok
        info = p.solver_info()
        p.close()
        return info, dx

    best = run()
    flat = _with_env("LBA_ND_LEVELS", "0", run)
    one = _with_env("LBA_ND_LEVELS", "1", run)
    assert flat[0]["levels"] == 0 and flat[0]["chain"] > best[0]["chain"]
    assert one[0]["levels"] <= 1
    for other in (flat, one):
        assert _rel(other[1], best[1]) <= 1e-8


def test_windows_without_a_loop_need_no_tail():
    for name in ("cfg1_local_50kf", "cfg0_cpu_plumbing"):
        p = Problem(make_config_window(name))
        assert p.solver_info()["tail"] == 0, name
        p.close()


def test_large_loop_band_solve():
    """700 keyframes around one loop (pose system 8400 > 6144: the substitution solve): normal equation
    residual against the oracle's system, LM descent, determinism."""
    win = make_window(n_opt_kf=699, n_fixed=1, n_lm=60000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True,
                      seed=13, loop=True, name="loop_700")
    o = orc.Oracle(win)
    chi_o, _, _ = o.errors()
    _, b_o, _ = o.build_system()
    p = Problem(win, early_stop=0)
    info = p.solver_info()
    assert info["band"] == 1 and info["chain"] < 0.75 * info["panels"]
    p.linearize()
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


def test_three_laps_window_revisits():
    win = make_window(**LAPS3)
    o = win.obs
    lap = np.minimum(o["kf_b"], 149) * 3 // 150
    seen = np.zeros((len(win.lm), 3), bool)
    seen[o["lm"], lap] = True
    assert (seen.sum(1) == 3).mean() > 0.5   # most landmarks are seen on every lap


@pytest.mark.parametrize("flags", [0, FLAG_BAND_SOLVE])
def test_three_laps_match_oracle(flags):
    """Two revisits of every place: the step and six LM iterations against the oracle; the graph
    dissection's chain at most 0.7 of the panels (every lap couples every other one: the interval
    dissection cannot cut the laps apart) with the same step."""
    win = make_window(**LAPS3)
    o = orc.Oracle(win)
    H_o, b_o, _ = o.build_system()
    lam = win.cfg["lambda_init"]
    ok_o, dx_o = o.solve(lam)
    p = Problem(win, flags=flags)
    info = p.solver_info()
    print("three laps:", info, "flops", p.solver_flops())
    assert info["chain"] <= 0.7 * info["panels"] and info["levels"] >= 2
    assert info["fill"] == info["tiles"] - info["s_tiles"] and info["fill"] >= 0
    res, H, b, _ = p.linearize()
    assert _rel(H, H_o) < 1e-9 and _rel(b, b_o) < 1e-9
    ok, dx = p.solve_step(lam)
    assert ok and ok_o
    n = p.pose_dim
    assert _rel(dx[:n], dx_o[:n]) <= 1e-6 and _rel(dx[n:], dx_o[n:]) <= 1e-6
    r = o.normal_residual(lam, dx)
    assert np.abs(r).max() <= 1e-8 * np.abs(b_o).max()

    def interval_only():
        q = Problem(win, flags=flags)
        q.linearize()
        ok2, dx2 = q.solve_step(lam)
        assert ok2
        return q.solver_info(), dx2

    info_iv, dx_iv = _with_env("LBA_ND_METHOD", "1", interval_only)
    assert info_iv["chain"] > info["chain"]
    assert _rel(dx_iv, dx) <= 1e-8
    o2 = orc.Oracle(win, early_stop=0)
    n_o, st_o = o2.optimize(6)
    p2 = Problem(win, early_stop=0, flags=flags)
    n2, st = p2.optimize(6)
    assert n2 == n_o and st.trials == st_o.trials
    assert abs(st.chi2_final - st_o.chi2_final) <= 1e-7 * st_o.chi2_final
    kf, lm = p2.state()
    kf_o, lm_o = o2.state()
    assert _rel(kf["t"], kf_o["t"]) <= 1e-6 and _rel(lm, lm_o) <= 1e-6
