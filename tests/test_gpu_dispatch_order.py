"""The workgroup dispatch orders are scheduling only: k_lin_schur's tiles longest first and k_assemble's S blocks
largest first (lba_host.hip tile_perm / asm_list) give bitwise the same LM run as index order
(LBA_DISPATCH_INDEX_ORDER), because every output is a fixed-order sum per tile / block."""
import os

import numpy as np
import pytest

from amc_lba import Problem
from amc_lba.synth import make_config_window, make_window


def _run(win, index_order):
    if index_order:
        os.environ["LBA_DISPATCH_INDEX_ORDER"] = "1"
    try:
        p = Problem(win, early_stop=0)   # (the orders are fixed at set-up)
    finally:
        os.environ.pop("LBA_DISPATCH_INDEX_ORDER", None)
    n, st = p.optimize(6)
    kf, lm = p.state()
    p.close()
    return n, st, kf, lm


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg0_cpu_plumbing", "loop", "cfg1_local_50kf"])
def test_dispatch_order_is_bitwise_neutral(name):
    win = make_window(n_opt_kf=24, n_lm=900, seed=5, loop=True) if name == "loop" else make_config_window(name)
    a = _run(win, False)
    b = _run(win, True)
    assert a[0] == b[0]
    assert (a[1].iterations, a[1].trials) == (b[1].iterations, b[1].trials)
    assert a[1].chi2_final == b[1].chi2_final and a[1].lambda_final == b[1].lambda_final
    for f in ("q", "t", "vel"):
        assert np.array_equal(a[2][f], b[2][f])
    assert np.array_equal(a[3], b[3])
