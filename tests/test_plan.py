"""Ordering and symbolic factorisation of the reduced camera system (amc-slam_amd/csrc/lba_plan.hpp, the
replacement of LinearSolverEigen's AMD-ordered SimplicialLDLT, Thirdparty/g2o/g2o/solvers/
linear_solver_eigen.h:60-124, at 32-row panel granularity), on the host: the order is a permutation with
the extrinsic panels last, the stored tiles of L are exactly the fill of a boolean elimination of the
permuted pattern, the update order is topological, and the dependent chain of band, loop-closure and
multi-revisit patterns is far below the panel count."""
import ctypes

import numpy as np
import pytest

I = ctypes.POINTER(ctypes.c_int)


def _p(a):
    return a.ctypes.data_as(I)


def plan(h, NP, pairs, NPk=None, levels=64, tail=True, method=0):
    NPk = NP if NPk is None else NPk
    pr = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1, 2))
    info = np.zeros(4, np.int32)
    ppos, uord = np.zeros(NP, np.int32), np.zeros(NP, np.int32)
    rowptr = np.zeros(NP + 1, np.int32)
    cap = NP * NP
    cols = np.zeros(cap, np.int32)
    nt = h.plan_probe(NP, NPk, len(pr), _p(pr), levels, int(tail), method, _p(info), _p(ppos), _p(uord), _p(rowptr),
                      _p(cols), cap)
    assert nt == info[3] >= NP
    return dict(chain=int(info[0]), tail=int(info[1]), levels=int(info[2]), ntile=int(nt), ppos=ppos, uord=uord,
                rowptr=rowptr, cols=cols[:nt])


def band_pairs(NP, w):
    return [(P, Q) for P in range(NP) for Q in range(max(0, P - w + 1), P)]


def revisit_pairs(NP, w, laps):
    """Panels of a trajectory of `laps` laps: a panel couples every panel within w of its position on
    the lap, on any lap (a place revisited laps - 1 times)."""
    per = NP / laps
    pos = np.arange(NP) % per
    d = np.abs(pos[:, None] - pos[None, :])
    d = np.minimum(d, per - d)
    P, Q = np.nonzero(np.tril(d < w, -1))
    return np.stack([P, Q], 1)


def check_plan(NP, pairs, pl, NPk=None):
    NPk = NP if NPk is None else NPk
    ppos = pl["ppos"]
    assert sorted(ppos.tolist()) == list(range(NP))
    assert sorted(pl["uord"].tolist()) == list(range(NP))
    assert all(ppos[P] == P for P in range(NPk, NP))   # extrinsic panels last, in order
    # boolean elimination of the permuted pattern
    M = np.eye(NP, dtype=bool)
    for P, Q in pairs:
        i, j = ppos[P], ppos[Q]
        M[max(i, j), min(i, j)] = True
    for j in range(NP):
        rows = j + 1 + np.nonzero(M[j + 1:, j])[0]
        if rows.size:
            M[np.ix_(rows, rows)] |= np.tril(np.ones((rows.size, rows.size), bool))
    L = np.tril(M)
    got = np.zeros((NP, NP), bool)
    for i in range(NP):
        cs = pl["cols"][pl["rowptr"][i]:pl["rowptr"][i + 1]]
        assert cs[-1] == i and np.all(np.diff(cs) > 0) if cs.size > 1 else cs[-1] == i
        got[i, cs] = True
    np.testing.assert_array_equal(got, L)
    # elimination-tree depth = reported chain; the update order is topological
    rank = np.empty(NP, int)
    rank[pl["uord"]] = np.arange(NP)
    depth = np.ones(NP, int)
    for j in range(NP):
        below = np.nonzero(L[j + 1:, j])[0]
        if below.size:
            par = j + 1 + below[0]
            depth[par] = max(depth[par], depth[j] + 1)
            assert np.all(rank[j + 1 + below] > rank[j])
    assert depth.max() == pl["chain"]


@pytest.mark.parametrize("NP,w", [(19, 5), (60, 3), (188, 4), (300, 2)])
def test_band(plan_harness, NP, w):
    pr = band_pairs(NP, w)
    pl = plan(plan_harness, NP, pr)
    check_plan(NP, pr, pl)
    assert pl["tail"] == 0
    if NP >= 60:
        assert pl["chain"] <= NP // 3 and pl["levels"] >= 2, pl["chain"]
    nat = plan(plan_harness, NP, pr, levels=0)
    check_plan(NP, pr, nat)
    assert nat["chain"] == NP and nat["ntile"] == sum(min(P + 1, w) for P in range(NP))


@pytest.mark.parametrize("laps", [1, 2, 3, 4])
def test_revisits(plan_harness, laps):
    """One loop closure (laps=1: the end meets the start) and two or three revisits of the same places:
    the interval dissection of the time order cannot separate laps that couple each other, the graph
    dissection (breadth-first level structures) can; the plan keeps the shorter chain."""
    NP, w = 240, 3
    pr = revisit_pairs(NP, w, laps)
    pl = plan(plan_harness, NP, pr)
    check_plan(NP, pr, pl)
    g = plan(plan_harness, NP, pr, method=2)
    iv = plan(plan_harness, NP, pr, method=1)
    check_plan(NP, pr, g)
    check_plan(NP, pr, iv)
    assert pl["chain"] == min(g["chain"], iv["chain"])
    assert pl["chain"] <= NP // 3, (pl["chain"], g["chain"], iv["chain"])
    if laps >= 3:
        assert g["chain"] < iv["chain"]


def test_extrinsic_panels_last(plan_harness):
    NP, NPk = 70, 66
    pr = band_pairs(NPk, 3) + [(P, Q) for P in range(NPk, NP) for Q in range(P)]
    for method in (0, 1, 2):
        pl = plan(plan_harness, NP, pr, NPk=NPk, method=method)
        check_plan(NP, pr, pl, NPk=NPk)


def test_random_sparse(plan_harness):
    rng = np.random.default_rng(3)
    for NP in (40, 120):
        pr = band_pairs(NP, 2) + [tuple(sorted(rng.choice(NP, 2, replace=False)))[::-1] for _ in range(NP // 8)]
        pl = plan(plan_harness, NP, pr)
        check_plan(NP, pr, pl)
