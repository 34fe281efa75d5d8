"""Window farm (BASELINE config 3) on one GPU: two windows cut from one trajectory,
each its own problem, exchanging their shared keyframes / landmarks through the engine
(lba_set_farm_group + lba_farm_plan + lba_farm_exchange: pack kernel, all-gather over an in-process
group, unpack kernel), compared with the same two windows optimised on the oracle and exchanged on
the host (amc_lba.farm.publish_owners decides the owners; the reference runs one LocalGPBA at a time
over the shared map, src/LocalMapping.cc:131, src/Optimizer.cc:1380-1432)."""
import dataclasses
import threading

import numpy as np
import pytest

import orc
from amc_lba import Group, Problem, farm

pytestmark = pytest.mark.gpu

SHAPE = dict(n_opt_kf=12, n_fixed=1, n_lm=1500, obs_per_lm=5, n_cam=2, gp=True)
STRIDE = 6


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
        t.join(timeout=300)
    if errs:
        raise errs[0]


def _host_exchange(wins, infos, states):
    """The owners' estimates into every other window (by global id), on the host."""
    out = [(k.copy(), l.copy()) for k, l in states]
    for r, (w, info) in enumerate(zip(wins, infos)):
        kfo, lmo = farm.publish_owners(info)
        for i in np.nonzero((lmo >= 0) & (lmo != r))[0]:
            o = lmo[i]
            j = int(np.searchsorted(wins[o].lm_gid, w.lm_gid[i]))
            out[r][1][i] = states[o][1][j]
        for i in np.nonzero((kfo >= 0) & (kfo != r))[0]:
            o = kfo[i]
            j = int(np.searchsorted(wins[o].kf_gid, w.kf_gid[i]))
            for f in ("q", "t", "vel"):
                out[r][0][f][i] = states[o][0][f][j]
    return out


@pytest.mark.parametrize("config,seed,stride", [(SHAPE, 5, STRIDE), ("cfg1_local_50kf", 20250912, 25)],
                         ids=["small", "cfg1_windows"])
def test_farm_two_windows_exchange_matches_oracle(config, seed, stride):
    """small: 12-KF windows; cfg1_windows: BASELINE config 3's per-rank shape (two config-1 windows,
    50 optimisable KFs each, stride 25 so neighbours share half their keyframes and landmarks)."""
    wins, infos = farm.make_farm_windows(config, 2, seed=seed, stride=stride)
    assert all((np.diff(w.lm_gid) > 0).all() and (np.diff(w.kf_gid) > 0).all() for w in wins)
    g = Group(2)
    probs = [Problem(w, early_stop=0) for w in wins]
    for r, p in enumerate(probs):
        p.set_farm_group(g, r)
    counts = [None, None]
    _threads(lambda r: counts.__setitem__(r, probs[r].farm_plan(wins[r].kf_gid, farm.publish_owners(infos[r])[0],
                                                                 wins[r].lm_gid, farm.publish_owners(infos[r])[1])), 2)
    # rank 0 owns every shared vertex (the lowest rank holding it): it publishes, rank 1 receives
    assert counts[0][0] > 0 and counts[0][1] > 0
    assert counts[0][2] == 0 and counts[0][3] == 0 and counts[1][0] == 0 and counts[1][1] == 0
    assert counts[1][2] == counts[0][0] and counts[1][3] == counts[0][1] and counts[0][4] == counts[1][4] == 0

    oracle_states = []
    for r in range(2):
        n, _ = probs[r].optimize(3)
        o = orc.Oracle(wins[r], early_stop=0)
        n_o, _ = o.optimize(3)
        assert n == n_o
        oracle_states.append(o.state())
    _threads(lambda r: probs[r].farm_exchange(), 2)
    gpu = [p.state() for p in probs]
    # bit-exact copies of the owner's estimates
    for i in np.nonzero(farm.publish_owners(infos[1])[1] == 0)[0]:
        j = int(np.searchsorted(wins[0].lm_gid, wins[1].lm_gid[i]))
        assert np.array_equal(gpu[1][1][i], gpu[0][1][j])
    for i in np.nonzero(farm.publish_owners(infos[1])[0] == 0)[0]:
        j = int(np.searchsorted(wins[0].kf_gid, wins[1].kf_gid[i]))
        for f in ("q", "t", "vel"):
            assert np.array_equal(gpu[1][0][f][i], gpu[0][0][f][j])
    # the oracle, exchanged on the host, then both sides optimise again from the exchanged estimates
    ex = _host_exchange(wins, infos, oracle_states)
    for r in range(2):
        k_o, l_o = ex[r]
        np.testing.assert_allclose(gpu[r][1], l_o, rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(gpu[r][0]["t"], k_o["t"], rtol=1e-6, atol=1e-6)
        n, st = probs[r].optimize(3)
        w2 = dataclasses.replace(wins[r], kfs=k_o, lm=l_o)
        o2 = orc.Oracle(w2, early_stop=0)
        n_o, st_o = o2.optimize(3)
        assert n == n_o
        assert abs(st.chi2_final - st_o.chi2_final) <= 1e-6 * st_o.chi2_final
        k2, l2 = probs[r].state()
        k2o, l2o = o2.state()
        np.testing.assert_allclose(l2, l2o, rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(k2["t"], k2o["t"], rtol=1e-6, atol=1e-6)
    for p in probs:
        p.close()
    g.close()


def test_farm_plan_requires_problem_and_collective():
    wins, infos = farm.make_farm_windows(SHAPE, 2, seed=5, stride=STRIDE)
    p = Problem(wins[0], early_stop=0)
    with pytest.raises(Exception):
        p.farm_exchange()   # no plan
    p.close()
