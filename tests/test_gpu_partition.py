"""Partitioned global BA (BASELINE config 4) on one GPU: the landmarks of a window
split over 2-3 ranks of an in-process all-reduce group (lba_group, the same engine path as the
RCCL ranks of a multi-GPU run: per trial one all-reduce of the reduced system and one of the trial
sums).  The ranks must take the LM decisions of the unpartitioned problem and end in its state."""
import threading

import numpy as np
import pytest

import orc
from amc_lba import Group, LbaError, Problem
from amc_lba.abi import FLAG_BAND_SOLVE
from amc_lba.gba import partition_window
from amc_lba.synth import make_window

pytestmark = pytest.mark.gpu

WINDOWS = {
    "global_shape": dict(n_opt_kf=11, n_fixed=1, n_lm=500, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=5),
    "global_mid": dict(n_opt_kf=99, n_fixed=1, n_lm=8000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, seed=6),
}


def _threads(fn, n):
    errs = []

    def wrap(r):
        try:
            fn(r)
        except Exception as e:   # noqa: BLE001 (re-raised below)
            errs.append(e)
    ts = [threading.Thread(target=wrap, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    if errs:
        raise errs[0]


def run_partitioned(win, nranks, iters, **over):
    g = Group(nranks)
    parts = [partition_window(win, r, nranks) for r in range(nranks)]
    probs = [None] * nranks
    _threads(lambda r: probs.__setitem__(r, Problem(parts[r][0], group=g, rank=r, early_stop=0, **over)), nranks)
    res = [None] * nranks
    _threads(lambda r: res.__setitem__(r, probs[r].optimize(iters)), nranks)
    states = [p.state() for p in probs]
    lm = np.zeros_like(win.lm)
    for (part, ids), (_, l) in zip(parts, states):
        lm[ids] = l
    for p in probs:
        p.close()
    g.close()
    return res, [s[0] for s in states], lm


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("name", list(WINDOWS))
@pytest.mark.parametrize("flags", [0, FLAG_BAND_SOLVE])
def test_partitioned_matches_single(name, nranks, flags):
    win = make_window(**WINDOWS[name])
    res, kfs, lm = run_partitioned(win, nranks, 6, flags=flags)
    p = Problem(win, early_stop=0, flags=flags)
    n1, st1 = p.optimize(6)
    kf1, lm1 = p.state()
    for (n, st), kf in zip(res, kfs):
        assert n == n1 and st.trials == st1.trials and st.result == st1.result
        assert abs(st.chi2_initial - st1.chi2_initial) <= 1e-11 * st1.chi2_initial
        assert abs(st.chi2_final - st1.chi2_final) <= 1e-9 * st1.chi2_final
        # every rank holds bitwise the same keyframe states (identical all-reduced systems)
        np.testing.assert_array_equal(kf["t"], kfs[0]["t"])
        np.testing.assert_array_equal(kf["q"], kfs[0]["q"])
    assert np.abs(kfs[0]["t"] - kf1["t"]).max() <= 1e-8 * np.abs(kf1["t"]).max()
    assert np.abs(lm - lm1).max() <= 1e-8 * np.abs(lm1).max()
    # and the oracle on the whole window
    o = orc.Oracle(win, early_stop=0)
    n_o, st_o = o.optimize(6)
    kf_o, lm_o = o.state()
    assert n_o == res[0][0] and st_o.trials == res[0][1].trials
    assert np.abs(lm - lm_o).max() <= 1e-6 * np.abs(lm_o).max()


def test_partitioned_needs_user_lambda():
    win = make_window(**WINDOWS["global_shape"])
    with pytest.raises(LbaError):
        run_partitioned(win, 2, 2, lambda_init=0.0)


def test_one_failing_rank_releases_its_peers():
    """A set-up that fails on one rank only (here an out-of-range observation in rank 1's partition)
    fails on every rank instead of leaving the others in the union-envelope all-reduce: the ranks
    exchange their set-up status first (partition status before the first collective)."""
    from dataclasses import replace
    from amc_lba.abi import LBA_E_ARG
    win = make_window(**WINDOWS["global_shape"])
    parts = [partition_window(win, r, 2)[0] for r in range(2)]
    bad = replace(parts[1], obs=parts[1].obs.copy())
    bad.obs["lm"][0] = len(bad.lm) + 5
    parts[1] = bad
    g = Group(2)
    codes = [None, None]

    def setup(r):
        try:
            Problem(parts[r], group=g, rank=r, early_stop=0).close()
            codes[r] = 0
        except LbaError as e:
            codes[r] = e.code
    ts = [threading.Thread(target=setup, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a rank hung in the set-up"
    g.close()
    assert codes == [LBA_E_ARG, LBA_E_ARG]


# ---- distributed factorisation (LBA_FLAG_SUBTREE_SOLVE): each rank factors its subtree of the nested
# dissection, the ranks sum their contributions to the top, every rank factors the top
LOOP_WINDOW = dict(n_opt_kf=199, n_fixed=1, n_lm=8000, obs_per_lm=6, n_cam=4, gp=True, global_ba=True, loop=True,
                   seed=7)


def run_split(win, nranks, iters, flags=0, **over):
    """The window split by lba_partition_assign over an in-process group; the ranks' states gathered (a
    keyframe from the rank whose subtree holds it, the top's from rank 0 after checking every rank agrees)."""
    import amc_lba
    from amc_lba.abi import FLAG_SUBTREE_SOLVE
    assign = amc_lba.partition_assign(win, nranks)
    g = Group(nranks)
    parts = [partition_window(win, r, nranks, assign) for r in range(nranks)]
    probs = [None] * nranks
    _threads(lambda r: probs.__setitem__(r, Problem(parts[r][0], group=g, rank=r, early_stop=0,
                                                    flags=FLAG_SUBTREE_SOLVE | flags, **over)), nranks)
    res = [None] * nranks
    _threads(lambda r: res.__setitem__(r, probs[r].optimize(iters)), nranks)
    states = [p.state() for p in probs]
    owners = [p.kf_owner() for p in probs]
    infos = [p.solver_info() for p in probs]
    for p in probs:
        p.close()
    g.close()
    own = owners[0]
    for o in owners[1:]:
        np.testing.assert_array_equal(o, own)   # every rank derives the same split
    kf = states[0][0].copy()
    top = own < 0
    for r in range(nranks):
        kr = states[r][0]
        np.testing.assert_array_equal(kr["q"][top], kf["q"][top])   # the top: bitwise the same on every rank
        np.testing.assert_array_equal(kr["t"][top], kf["t"][top])
        kf[own == r] = kr[own == r]
    lm = np.zeros_like(win.lm)
    for (part, ids), (_, l) in zip(parts, states):
        lm[ids] = l
    return res, kf, lm, own, infos


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("name", ["global_mid", "loop"])
def test_subtree_solve_matches_single(name, nranks):
    win = make_window(**(LOOP_WINDOW if name == "loop" else WINDOWS[name]))
    res, kf, lm, own, infos = run_split(win, nranks, 6)
    assert (own >= 0).sum() > 0 and len(set(own[own >= 0])) == nranks, own   # every rank owns a subtree
    p = Problem(win, early_stop=0, flags=FLAG_BAND_SOLVE)
    n1, st1 = p.optimize(6)
    kf1, lm1 = p.state()
    p.close()
    for n, st in res:
        assert n == n1 and st.trials == st1.trials and st.result == st1.result
        assert abs(st.chi2_initial - st1.chi2_initial) <= 1e-11 * st1.chi2_initial
        assert abs(st.chi2_final - st1.chi2_final) <= 1e-9 * st1.chi2_final
    assert np.abs(kf["t"] - kf1["t"]).max() <= 1e-8 * np.abs(kf1["t"]).max()
    assert np.abs(kf["vel"] - kf1["vel"]).max() <= 1e-7 * max(np.abs(kf1["vel"]).max(), 1.0)
    assert np.abs(lm - lm1).max() <= 1e-8 * np.abs(lm1).max()


def test_subtree_solve_one_step_matches_single():
    """One LM iteration (one damped solve) of the distributed factorisation against the unpartitioned
    problem's: the step agrees to 1e-9 (only the summation order of the top's contributions differs)."""
    win = make_window(**WINDOWS["global_mid"])
    x0 = win.kfs.copy()
    res, kf, lm, own, _ = run_split(win, 2, 1)
    p = Problem(win, early_stop=0, flags=FLAG_BAND_SOLVE)
    p.optimize(1)
    kf1, lm1 = p.state()
    p.close()
    dt, dt1 = kf["t"] - x0["t"], kf1["t"] - x0["t"]
    assert np.abs(dt - dt1).max() <= 1e-9 * np.abs(dt1).max()
    dl, dl1 = lm - win.lm, lm1 - win.lm
    assert np.abs(dl - dl1).max() <= 1e-9 * np.abs(dl1).max()


def test_subtree_solve_rejects_a_stray_landmark():
    """A rank holding a landmark of another rank's subtree (the replicated solve's l % N split) fails its
    set-up on every rank instead of factoring a wrong system."""
    from amc_lba.abi import FLAG_SUBTREE_SOLVE, LBA_E_ARG
    win = make_window(**WINDOWS["global_mid"])
    parts = [partition_window(win, r, 2)[0] for r in range(2)]   # (not lba_partition_assign's split)
    g = Group(2)
    codes = [None, None]

    def setup(r):
        try:
            Problem(parts[r], group=g, rank=r, early_stop=0, flags=FLAG_SUBTREE_SOLVE).close()
            codes[r] = 0
        except LbaError as e:
            codes[r] = e.code
    ts = [threading.Thread(target=setup, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a rank hung in the set-up"
    g.close()
    assert codes == [LBA_E_ARG, LBA_E_ARG]
