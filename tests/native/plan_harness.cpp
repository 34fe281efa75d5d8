// Host build of the reduced camera system's ordering and symbolic factorisation (amc-slam_amd/csrc/
// lba_plan.hpp, the header lba_set_problem uses) for the CPU tests: tests/test_plan.py checks the order
// is a permutation, the stored tiles are exactly the fill of a boolean elimination of the permuted
// pattern, the update order is topological, and the chain of band / loop / multi-revisit patterns.
#include <cstring>
#include <vector>

#include "../../amc-slam_amd/csrc/lba_plan.hpp"

extern "C" {

// pairs: npairs (P, Q) panel couplings (any order; the diagonal is implied).  info: chain, tail, levels,
// ntile.  ppos[NP], uord[NP], rowptr[NP + 1] and cols[cap] receive the plan.  Returns ntile, or -1 when
// cap is too small.
static std::vector<std::vector<int>> lower_of(int NP, int npairs, const int* pairs) {
    std::vector<std::vector<int>> lower(NP);
    for (int P = 0; P < NP; ++P) lower[P].push_back(P);
    for (int k = 0; k < npairs; ++k) {
        const int a = pairs[2 * k], b = pairs[2 * k + 1];
        lower[a > b ? a : b].push_back(a > b ? b : a);
    }
    for (auto& l : lower) {
        std::sort(l.begin(), l.end());
        l.erase(std::unique(l.begin(), l.end()), l.end());
    }
    return lower;
}

int plan_probe(int NP, int NPk, int npairs, const int* pairs, int max_levels, int tail_search, int method, int* info,
               int* ppos, int* uord, int* rowptr, int* cols, int cap) {
    const auto lower = lower_of(NP, npairs, pairs);
    const lba_plan::Plan pl = lba_plan::make_plan(NP, NPk, lower, max_levels, tail_search != 0, 16, method);
    info[0] = pl.chain;
    info[1] = pl.tail;
    info[2] = pl.levels;
    info[3] = pl.ntile();
    if (pl.ntile() > cap) return -1;
    std::memcpy(ppos, pl.ppos.data(), sizeof(int) * NP);
    std::memcpy(uord, pl.uord.data(), sizeof(int) * NP);
    std::memcpy(rowptr, pl.rowptr.data(), sizeof(int) * (NP + 1));
    std::memcpy(cols, pl.cols.data(), sizeof(int) * pl.ntile());
    return pl.ntile();
}

// The distributed factorisation's split (lba_plan::split_subtrees) of the plan make_plan makes (the arguments
// lba_set_problem / lba_partition_assign pass: 64 levels, tail search on, both methods): own[NP] the rank of
// each factorisation position's subtree (-1 the top), parent[NP] its elimination-tree parent (-1 a root).
// Returns the number of tiles of L.
int split_probe(int NP, int NPk, int npairs, const int* pairs, int nranks, int* own, int* parent) {
    const auto lower = lower_of(NP, npairs, pairs);
    const lba_plan::Plan pl = lba_plan::make_plan(NP, NPk, lower, 64, true, 16, 0);
    const std::vector<int> o = lba_plan::split_subtrees(pl, nranks);
    for (int j = 0; j < NP; ++j) {
        own[j] = o[j];
        parent[j] = pl.colrows[j].empty() ? -1 : pl.colrows[j].front();
    }
    return pl.ntile();
}
}
