"""Tracking-side pose optimisation on the GPU (lba_track: Optimizer::PoseGPOptimizationFromeLastFrame,
src/Optimizer.cc:369-686) against the oracle's restatement (orc_track_pose) frame by frame: the same
outlier classification, return value and iteration count, the optimised pose within the north-star
pose tolerance.  A batch mixes fixed and free previous frames and runs as one launch."""
import numpy as np
import pytest

import orc
from amc_lba import LbaError
from amc_lba.synth import make_window
from amc_lba.track import Tracker, make_track_frames, track_config

pytestmark = pytest.mark.gpu


def _batch():
    frames, obs = [], []
    for seed, ks, fix in ((4, [3, 6, 9, 12], True), (7, [2, 5, 8, 11], False)):
        win = make_window(n_opt_kf=12, n_fixed=1, n_lm=3000, obs_per_lm=6, n_cam=4, gp=True, seed=seed, perturb=False)
        f, o = make_track_frames(win, ks, fix_prev=fix, seed=seed)
        f["obs0"] += sum(len(x) for x in obs)
        frames.append(f)
        obs.append(o)
    return np.concatenate(frames), np.concatenate(obs), win.cams


def test_track_batch_matches_oracle():
    frames, obs, cams = _batch()
    cfg = track_config()
    fr_g, ob_g = Tracker(cfg).track(frames.copy(), obs.copy(), cams)
    for f in range(len(frames)):
        a = frames[f:f + 1].copy()
        s = slice(frames[f]["obs0"], frames[f]["obs0"] + frames[f]["n_obs"])
        o = obs[s].copy()
        n_o = orc.track_pose(cfg, a, o, cams)
        g = fr_g[f]
        assert g["n_good"] == n_o and g["iterations"] == a[0]["iterations"], f
        np.testing.assert_array_equal(ob_g["outlier"][s], o["outlier"], err_msg=f"frame {f}")
        assert np.abs(g["cur"]["t"] - a[0]["cur"]["t"]).max() <= 1e-6 * max(1.0, np.abs(a[0]["cur"]["t"]).max())
        qg = g["cur"]["q"] * np.sign(g["cur"]["q"][3])
        qo = a[0]["cur"]["q"] * np.sign(a[0]["cur"]["q"][3])
        assert np.abs(qg - qo).max() <= 1e-7
        assert np.abs(g["cur"]["vel"] - a[0]["cur"]["vel"]).max() <= 1e-5
        # the previous frame is never written back; the optimisation moved towards the truth
        np.testing.assert_array_equal(g["prev"]["t"], frames[f]["prev"]["t"])
    assert (fr_g["n_good"] > 0.8 * fr_g["n_obs"]).all()


def test_track_small_frame_stops_after_one_round():
    frames, obs, cams = _batch()
    f = frames[:1].copy()
    o = obs[: 5].copy()
    f["n_obs"] = 5
    cfg = track_config()
    fg, og = Tracker(cfg).track(f.copy(), o.copy(), cams)
    a = f.copy()
    oo = o.copy()
    n_o = orc.track_pose(cfg, a, oo, cams)
    assert fg[0]["n_good"] == n_o and fg[0]["iterations"] == a[0]["iterations"] <= 10
    np.testing.assert_array_equal(og["outlier"], oo["outlier"])


def test_track_rejects_bad_input():
    frames, obs, cams = _batch()
    t = Tracker(track_config())
    bad = obs.copy()
    bad["kind"][0] = 7
    with pytest.raises(LbaError):
        t.track(frames, bad, cams)
    f = frames.copy()
    f["cur"]["time"] = f["prev"]["time"]
    with pytest.raises(LbaError):
        t.track(f, obs, cams)
