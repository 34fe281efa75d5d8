// Randomised equivalence check of make_plan's loop-closure tail search (lba_plan.hpp): the original per-(c, a)
// downward scan against the O(NP^2) running-max form adopted in round 3.  g++ -O2 tail_search_eq.cpp && ./a.out
#include <vector>
#include <cstdio>
#include <random>
#include <algorithm>
int old_best(const std::vector<int>& pfirst, int NPk, int NP) {
    int c_best = NPk, bestlen = NP + 1;
    for (int c = NPk; c >= 1; --c) {
        if (NPk - c >= bestlen) break;
        for (int a = 1; a < c; ++a) {
            int b = c;
            while (b > a && pfirst[b - 1] >= a) --b;
            if (b >= c) continue;
            const int len = std::max(a, c - b) + (b - a) + (NPk - c);
            if (len < bestlen) { bestlen = len; c_best = c; }
        }
    }
    if (bestlen > NPk) c_best = NPk;
    return c_best * 100000 + bestlen;
}
int new_best(const std::vector<int>& pfirst, int NPk, int NP) {
    int c_best = NPk, bestlen = NP + 1;
    std::vector<int> mv(NP + 1);
    for (int c = NPk; c >= 1; --c) {
        if (NPk - c >= bestlen) break;
        std::fill(mv.begin(), mv.begin() + c, -1);
        for (int r = 0; r < c; ++r) mv[pfirst[r]] = std::max(mv[pfirst[r]], r);
        int M = -1;
        for (int a = 1; a < c; ++a) {
            M = std::max(M, mv[a - 1]);
            const int b = M >= a ? M + 1 : a;
            if (b >= c) continue;
            const int len = std::max(a, c - b) + (b - a) + (NPk - c);
            if (len < bestlen) { bestlen = len; c_best = c; }
        }
    }
    if (bestlen > NPk) c_best = NPk;
    return c_best * 100000 + bestlen;
}
int main() {
    std::mt19937 g(7);
    int bad = 0;
    for (int it = 0; it < 20000; ++it) {
        int NP = 1 + g() % 60, NPk = 1 + g() % NP;
        std::vector<int> pf(NP);
        int band = 1 + g() % 6;
        for (int P = 0; P < NP; ++P) {
            int f = std::max(0, P - (int)(g() % (band + 1)));
            if (g() % 13 == 0) f = g() % (P + 1);   // loop closures
            pf[P] = f;
        }
        if (old_best(pf, NPk, NP) != new_best(pf, NPk, NP)) ++bad;
    }
    printf("mismatches %d\n", bad);
}
