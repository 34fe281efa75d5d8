"""make_plan's loop-closure tail search and split_subtrees (amc-slam_amd/csrc/lba_plan.hpp), host only, through
the header itself (tests/native/plan_harness.cpp):
- the tail make_plan picks (interval method) equals the original per-(c, a) downward scan, restated here, on
  random banded envelopes with loop-closure rows, and the tail's panels are ordered last;
- the distributed factorisation's split: disjoint subtrees that are closed under descendants, every coupled pair
  of L's columns inside one subtree or reaching the top, every rank given work, and the same split every time."""
import ctypes

import numpy as np
import pytest

from test_plan import band_pairs, plan, revisit_pairs

I = ctypes.POINTER(ctypes.c_int)


def _p(a):
    return a.ctypes.data_as(I)


def scan_tail(pfirst, NPk, NP):
    """The round-2 form of the search (a scan per (c, a)): c_best, the first panel of the tail."""
    c_best, bestlen = NPk, NP + 1
    for c in range(NPk, 0, -1):
        if NPk - c >= bestlen:
            break
        for a in range(1, c):
            b = c
            while b > a and pfirst[b - 1] >= a:
                b -= 1
            if b >= c:
                continue
            ln = max(a, c - b) + (b - a) + (NPk - c)
            if ln < bestlen:
                bestlen, c_best = ln, c
    return NPk if bestlen > NPk else c_best


def random_envelope(rng, NP):
    band = int(rng.integers(1, 7))
    pairs, pfirst = [], []
    for P in range(NP):
        f = max(0, P - int(rng.integers(0, band + 1)))
        if rng.integers(0, 13) == 0:
            f = int(rng.integers(0, P + 1))   # a loop closure
        pfirst.append(f)
        pairs += [(P, f)] if f < P else []
        pairs += [(P, Q) for Q in range(max(f + 1, P - band), P)]
    return pairs, pfirst


def test_tail_search_matches_scan(plan_harness):
    rng = np.random.default_rng(7)
    checked = 0
    for _ in range(600):
        NP = int(rng.integers(2, 50))
        pairs, _ = random_envelope(rng, NP)
        pfirst = list(range(NP))
        for P, Q in pairs:
            pfirst[P] = min(pfirst[P], Q)
        c = scan_tail(pfirst, NP, NP)
        pl = plan(plan_harness, NP, pairs, method=1)
        assert pl["tail"] == NP - c, (NP, pairs)
        # the tail's panels take the last positions, in natural order
        assert all(pl["ppos"][P] == P for P in range(c, NP))
        checked += c < NP
    assert checked > 20   # (some envelopes did take a tail)


def split(h, NP, pairs, nranks, NPk=None):
    NPk = NP if NPk is None else NPk
    pr = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1, 2))
    own, parent = np.zeros(NP, np.int32), np.zeros(NP, np.int32)
    nt = h.split_probe(NP, NPk, len(pr), _p(pr), nranks, _p(own), _p(parent))
    assert nt >= NP
    return own, parent


@pytest.mark.parametrize("NP,pairs", [(188, band_pairs(188, 4)), (300, band_pairs(300, 2)),
                                      (240, revisit_pairs(240, 3, 1)), (240, revisit_pairs(240, 3, 3))])
@pytest.mark.parametrize("nranks", [2, 3, 4, 8])
def test_split_subtrees(plan_harness, NP, pairs, nranks):
    own, parent = split(plan_harness, NP, pairs, nranks)
    own2, _ = split(plan_harness, NP, pairs, nranks)
    np.testing.assert_array_equal(own, own2)   # deterministic: every rank derives the same split
    assert own.min() >= -1 and own.max() < nranks
    assert set(own[own >= 0].tolist()) == set(range(nranks))   # every rank owns a subtree
    # closed under descendants: a subtree column's parent is in the same subtree or the top; a top column's
    # parent is in the top
    for j in range(NP):
        if parent[j] >= 0:
            assert own[parent[j]] in (own[j], -1), (j, own[j], own[parent[j]])
            if own[j] < 0:
                assert own[parent[j]] < 0
    # coupled columns (tile (i, j) of L non-zero) lie in one subtree, or the row is in the top
    pl = plan(plan_harness, NP, pairs)
    for i in range(NP):
        for j in pl["cols"][pl["rowptr"][i]:pl["rowptr"][i + 1]]:
            assert own[i] == own[j] or own[i] == -1, (i, j, own[i], own[j])
    # the top is small next to the subtrees
    assert (own < 0).sum() < NP // 4


def test_split_one_rank(plan_harness):
    own, _ = split(plan_harness, 60, band_pairs(60, 3), 1)
    assert np.all(own == 0)
