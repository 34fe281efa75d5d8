"""The round-4 launch fusions change no result bit: k_exp_asm (the pose samples' expansion and the assembly of S / b in
one launch, each output waiting only for its own samples) against k_expand + k_assemble (LBA_NO_FUSED_ASM), and the
trial evaluation inside k_update (tiles waiting for their samples' producers) against k_update + k_eval
(LBA_NO_FUSED_EVAL): the same LM runs, bitwise, in the device-decided (queued) loop and the host-driven loop."""
import os
from dataclasses import replace

import numpy as np
import pytest

from amc_lba import Problem
from amc_lba.abi import FLAG_HOST_LOOP, MONO, STEREO
from amc_lba.synth import make_config_window, make_window

pytestmark = pytest.mark.gpu


def _run(win, env, flags=0):
    os.environ.update(env)
    try:
        p = Problem(win, early_stop=0, flags=flags)   # (the fusions are chosen at set-up)
    finally:
        for k in env:
            os.environ.pop(k, None)
    n, st = p.optimize(6)
    kf, lm = p.state()
    p.close()
    return n, st, kf, lm


def _same(a, b):
    assert a[0] == b[0]
    assert (a[1].iterations, a[1].trials, a[1].solve_failures) == (b[1].iterations, b[1].trials, b[1].solve_failures)
    assert a[1].chi2_initial == b[1].chi2_initial
    assert a[1].chi2_final == b[1].chi2_final and a[1].lambda_final == b[1].lambda_final
    for f in ("q", "t", "vel"):
        assert np.array_equal(a[2][f], b[2][f])
    assert np.array_equal(a[3], b[3])


WINDOWS = {
    "gp_small": lambda: make_window(n_opt_kf=8, n_lm=600, obs_per_lm=6, n_cam=4, gp=True, seed=3),
    "mono_nogp": lambda: make_window(n_opt_kf=8, n_lm=600, obs_per_lm=6, n_cam=2, gp=False, seed=4),
    "cfg1": lambda: make_config_window("cfg1_local_50kf"),
}


@pytest.mark.parametrize("name", list(WINDOWS))
@pytest.mark.parametrize("flags", [0, FLAG_HOST_LOOP])
def test_fused_launches_are_bitwise_neutral(name, flags):
    win = WINDOWS[name]()
    fused = _run(win, {}, flags)
    _same(fused, _run(win, {"LBA_NO_FUSED_ASM": "1"}, flags))
    _same(fused, _run(win, {"LBA_NO_FUSED_EVAL": "1"}, flags))


def _many_kf_window():
    """4200 keyframes with their motion priors and velocity edges but no GP observation (so no GP pair workgroups:
    the fused k_update grid stays resident), few landmarks: the motion-prior items of the fused evaluation wait for
    66 KF blocks, more than one 64-lane round of producers (priors touching keyframes >= 4096)."""
    w = make_window(n_opt_kf=4200, n_lm=3000, obs_per_lm=6, n_cam=2, gp=True, seed=5, global_ba=True)
    keep = np.isin(w.obs["kind"], (MONO, STEREO))
    return replace(w, obs=np.ascontiguousarray(w.obs[keep]), name="kf4200")


@pytest.mark.parametrize("flags", [0, FLAG_HOST_LOOP])
def test_fused_eval_waits_for_every_kf_block(flags):
    win = _many_kf_window()
    p = Problem(win, early_stop=0, flags=flags)
    modes = p.kernel_modes()
    p.close()
    assert modes["fuse_eval"] == 1, modes   # (the case under test: the fused evaluation with > 64 KF blocks)
    fused = _run(win, {}, flags)
    _same(fused, _run(win, {"LBA_NO_FUSED_EVAL": "1"}, flags))


def test_fused_launches_repeatable_on_all_xcds():
    """The fused hand-offs (plain loads after relaxed flag polls, write-through stores before relaxed flag stores: the
    visibility argument of k_update / k_exp_asm) give the unfused results on a grid spread over all eight XCDs, run after
    run (a stress check of the protocol in place of acquire / release fences)."""
    win = WINDOWS["cfg1"]()
    ref = _run(win, {"LBA_NO_FUSED_ASM": "1", "LBA_NO_FUSED_EVAL": "1"})
    for _ in range(4):
        _same(ref, _run(win, {}))
