"""The bounded in-launch waits' failure path (LBA_E_TIMEOUT, include/amc_lba.h): a wait that gives up sets the
device fault word, and the call that reads it fails instead of returning results computed from data that may be
stale.  lba_debug_inject_fault sets the word as such a wait does, so every call that reads it is checked without a
hang: it fails with LBA_E_TIMEOUT, the word is cleared, and the next call (and a new set-up) run normally."""
import numpy as np
import pytest

from amc_lba import LbaError, Problem
from amc_lba.abi import LBA_E_TIMEOUT
from amc_lba.synth import make_window

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def win():
    return make_window(n_opt_kf=8, n_lm=600, seed=11)


@pytest.mark.parametrize("code", [1, 2, 4])
def test_injected_fault_fails_each_call_and_clears(win, code):
    ref = Problem(win, early_stop=0)
    n_ref, st_ref = ref.optimize(3)
    kf_ref, lm_ref = ref.state()
    ref.close()
    p = Problem(win, early_stop=0)
    calls = [lambda: p.optimize(3), lambda: p.solve_step(1e-3), lambda: p.linearize(), lambda: p.eval()]
    for call in calls:
        p.inject_fault(code)
        with pytest.raises(LbaError) as e:
            call()
        assert e.value.code == LBA_E_TIMEOUT
        assert "timed out" in str(e.value)
        call()   # the word was cleared: the same call runs
    # a new set-up of the same window reproduces the clean run bit for bit (counters, flags and state reset)
    p.close()
    p = Problem(win, early_stop=0)
    p.inject_fault(code)
    with pytest.raises(LbaError):
        p.optimize(3)
    p.close()
    p = Problem(win, early_stop=0)
    n, st = p.optimize(3)
    kf, lm = p.state()
    p.close()
    assert n == n_ref and st.trials == st_ref.trials and st.chi2_final == st_ref.chi2_final
    np.testing.assert_array_equal(kf["t"], kf_ref["t"])
    np.testing.assert_array_equal(lm, lm_ref)
