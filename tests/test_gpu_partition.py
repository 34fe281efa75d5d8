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
