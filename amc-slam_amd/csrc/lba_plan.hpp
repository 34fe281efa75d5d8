// lba_plan.hpp — host-side ordering and symbolic structure of the reduced camera system's factorisation
// (the replacement of LinearSolverEigen's AMD-ordered SimplicialLDLT, Thirdparty/g2o/g2o/solvers/
// linear_solver_eigen.h:60-124, at the granularity of 32-row panels).
//
// The pose system of a (local or global) BA is a band in time order (a landmark couples the keyframes
// that see it) plus, after loop closures, blocks between keyframes that revisit the same place.  The
// panels are ordered by nested dissection, planned two ways and the order with the shorter dependent
// chain kept:
//  - interval dissection of the time order: [left | separator | right] cuts with no row of the right
//    part coupling a column of the left part, recursively; rows that reach back across the whole window
//    (one loop closure: the last keyframes see the first ones' landmarks) are taken out first as a tail;
//  - graph dissection of the panel graph: separators from breadth-first level structures (George), which
//    cut a trajectory that revisits its places several times (every lap couples every other one) where
//    no interval of the time order separates anything.
// Both parts of a cut are ordered first (recursively), the separator after them; independent parts
// complete side by side (the update order interleaves them).  The panels of free extrinsics (dense
// rows) are ordered last.  The factorisation's dependent chain is then the depth of the elimination
// tree (leaf + separators) instead of every panel.
//
// The structure of L (which 32 x 32 tiles are non-zero, fill-in included) follows from a tile-level
// symbolic factorisation of the permuted pattern (the elimination-tree row merge), so the solver stores
// and touches only those tiles: with a dissection the envelope of the permuted matrix is far larger than
// its fill.
#pragma once

#include <algorithm>
#include <vector>

namespace lba_plan {

struct Plan {
    int NP = 0;
    int chain = 0;                          // panels on the dissection's dependent chain (estimate)
    int tail = 0;                           // panels of the loop-closure tail (ordered last)
    int levels = 0;                         // depth of the dissection tree
    std::vector<int> ppos, pnat;            // natural panel -> factorisation position, and back
    std::vector<int> uord, rank;            // positions in update (completion) order; each position's rank
    std::vector<int> rowptr, cols;          // tiles of L by row (positions), columns ascending, diagonal last
    std::vector<std::vector<int>> colrows;  // per column: the rows below the diagonal, ascending
    int ntile() const { return rowptr.empty() ? 0 : rowptr.back(); }
    int tile_id(int i, int j) const {       // -1 if (i, j) is structurally zero
        const int* b = cols.data() + rowptr[i];
        const int* e = cols.data() + rowptr[i + 1];
        const int* q = std::lower_bound(b, e, j);
        return (q != e && *q == j) ? (int)(q - cols.data()) : -1;
    }
    bool nz(int i, int j) const { return tile_id(i, j) >= 0; }
};

namespace detail {

struct Node {
    std::vector<int> order;   // natural panels in factorisation order
    std::vector<int> uord;    // natural panels in update order
    int chain = 0, depth = 0;
};

// merge two update orders side by side (left k and right k alternately): the two halves of a dissection
// complete concurrently
inline std::vector<int> interleave(const std::vector<int>& a, const std::vector<int>& b) {
    std::vector<int> o;
    o.reserve(a.size() + b.size());
    for (size_t k = 0; k < std::max(a.size(), b.size()); ++k) {
        if (k < a.size()) o.push_back(a[k]);
        if (k < b.size()) o.push_back(b[k]);
    }
    return o;
}

// nested dissection of the natural panel range [lo, hi); lower[P]: natural panels Q <= P coupled with P.
// mirror: the right part of every cut is ordered from its far end (desc: this range's leaves descending), so
// a leaf's columns next to the separator come last and only they take the separator's rows: with the
// separator's rows in every column of an ascending right part, the fill of a band of width w grows by
// about w tiles per column of that part (config 1: 120 -> 100 tiles of L)
inline Node dissect(int lo, int hi, const std::vector<std::vector<int>>& lower, int leaf, int max_depth, bool mirror = false,
                    bool desc = false) {
    Node n;
    const int len = hi - lo;
    auto as_leaf = [&]() {
        for (int P = lo; P < hi; ++P) n.order.push_back(desc ? lo + hi - 1 - P : P);
        n.uord = n.order;
        n.chain = len;
        n.depth = 0;
        return n;
    };
    if (len <= leaf || max_depth <= 0) return as_leaf();
    // lowc[P - lo]: the lowest panel of [lo, hi) that P couples with (P itself if none below)
    std::vector<int> lowc(len);
    for (int P = lo; P < hi; ++P) {
        int m = P;
        for (int Q : lower[P])
            if (Q >= lo && Q < m) m = Q;
        lowc[P - lo] = m;
    }
    // a separator [a, b): every row of [b, hi) couples only columns >= a.  last[a] = the last row of
    // [a, hi) with a coupling left of a: b(a) = last + 1.
    int best_a = -1, best_b = -1, best_cost = len;
    for (int a = lo + len / 4; a <= lo + (3 * len) / 4; ++a) {
        if (a <= lo) continue;
        int b = a + 1;
        for (int P = a; P < hi; ++P)
            if (lowc[P - lo] < a) b = std::max(b, P + 1);
        if (b >= hi) continue;
        const int cost = (b - a) + std::max(a - lo, hi - b);
        if (cost < best_cost) { best_cost = cost; best_a = a; best_b = b; }
    }
    if (best_a < 0 || best_cost >= len) return as_leaf();
    Node L = dissect(lo, best_a, lower, leaf, max_depth - 1, mirror, false);
    Node R = dissect(best_b, hi, lower, leaf, max_depth - 1, mirror, mirror);
    n.order = L.order;
    n.order.insert(n.order.end(), R.order.begin(), R.order.end());
    n.uord = interleave(L.uord, R.uord);
    for (int P = best_a; P < best_b; ++P) {
        n.order.push_back(P);
        n.uord.push_back(P);
    }
    n.chain = std::max(L.chain, R.chain) + (best_b - best_a);
    n.depth = 1 + std::max(L.depth, R.depth);
    return n;
}

// nested dissection of a general panel graph (adjacency adj, restricted to the vertices `vs`): the
// connected components are independent; a component is cut by a level of a breadth-first search from a
// pseudo-peripheral vertex (George's level structure): the level's vertices with a neighbour in the next
// level separate the levels below from the levels above.  For a band (the time order of a window) the
// levels are intervals of time and this is the interval cut of dissect(); for a trajectory that revisits
// its start (one or several loop closures) the levels are arcs of every lap at once, which no interval of
// the natural order separates.
inline Node dissect_graph(std::vector<int> vs, const std::vector<std::vector<int>>& adj, std::vector<int>& mark,
                          int& stamp, int leaf, int max_depth) {
    Node n;
    std::sort(vs.begin(), vs.end());
    auto as_leaf = [&]() {
        n.order = vs;
        n.uord = vs;
        n.chain = (int)vs.size();
        n.depth = 0;
        return n;
    };
    if ((int)vs.size() <= leaf || max_depth <= 0) return as_leaf();
    // mark[v] == in_set: v belongs to this call's vertex set (stamps are unique per call)
    const int in_set = ++stamp;
    for (int v : vs) mark[v] = in_set;
    std::vector<int> level(mark.size(), -1);
    // breadth-first levels from `root` inside the set; returns the levels, vertices in BFS order
    auto bfs = [&](int root, std::vector<int>& seen) {
        seen.clear();
        for (int v : vs) level[v] = -1;
        level[root] = 0;
        seen.push_back(root);
        for (size_t h = 0; h < seen.size(); ++h) {
            const int v = seen[h];
            for (int w : adj[v])
                if (mark[w] == in_set && level[w] < 0) { level[w] = level[v] + 1; seen.push_back(w); }
        }
    };
    std::vector<int> seen;
    bfs(vs.front(), seen);
    if (seen.size() < vs.size()) {   // several components: order them one after another, complete side by side
        std::vector<std::vector<int>> comps;
        std::vector<char> done(mark.size(), 0);
        for (int v : vs) {
            if (done[v]) continue;
            bfs(v, seen);
            for (int w : seen) done[w] = 1;
            comps.push_back(seen);
        }
        for (auto& c : comps) {
            Node m = dissect_graph(c, adj, mark, stamp, leaf, max_depth);
            n.order.insert(n.order.end(), m.order.begin(), m.order.end());
            n.uord = interleave(n.uord, m.uord);
            n.chain = std::max(n.chain, m.chain);
            n.depth = std::max(n.depth, m.depth);
        }
        return n;
    }
    // pseudo-peripheral root: repeat from the last level's lowest-degree vertex while the eccentricity grows
    int root = vs.front(), ecc = level[seen.back()];
    for (int it = 0; it < 4; ++it) {
        int best = seen.back(), bd = 1 << 30;
        for (int k = (int)seen.size() - 1; k >= 0 && level[seen[k]] == ecc; --k) {
            int d = 0;
            for (int w : adj[seen[k]]) d += mark[w] == in_set;
            if (d < bd) { bd = d; best = seen[k]; }
        }
        std::vector<int> s2;
        bfs(best, s2);
        const int e2 = level[s2.back()];
        if (e2 <= ecc) { bfs(root, seen); break; }
        root = best; ecc = e2; seen = s2;
    }
    if (ecc < 2) return as_leaf();
    std::vector<int> cnt(ecc + 1, 0), nsep(ecc + 1, 0);
    for (int v : vs) ++cnt[level[v]];
    for (int v : vs) {   // v separates if it has a neighbour one level up
        for (int w : adj[v])
            if (mark[w] == in_set && level[w] == level[v] + 1) { ++nsep[level[v]]; break; }
    }
    int best_s = -1;
    long best_cost = (long)vs.size();
    int below = 0;
    for (int l = 0; l <= ecc; ++l) {
        if (l >= 1 && l <= ecc - 1) {
            const int left = below + cnt[l] - nsep[l], right = (int)vs.size() - below - cnt[l];
            const long cost = nsep[l] + std::max(left, right);
            if (cost < best_cost) { best_cost = cost; best_s = l; }
        }
        below += cnt[l];
    }
    if (best_s < 0) return as_leaf();
    std::vector<int> A, B, S;
    for (int v : vs) {
        const int l = level[v];
        if (l < best_s) A.push_back(v);
        else if (l > best_s) B.push_back(v);
        else {
            bool up = false;
            for (int w : adj[v])
                if (mark[w] == in_set && level[w] == l + 1) { up = true; break; }
            (up ? S : A).push_back(v);
        }
    }
    Node L = dissect_graph(A, adj, mark, stamp, leaf, max_depth - 1);
    Node R = dissect_graph(B, adj, mark, stamp, leaf, max_depth - 1);
    n.order = L.order;
    n.order.insert(n.order.end(), R.order.begin(), R.order.end());
    n.uord = interleave(L.uord, R.uord);
    std::sort(S.begin(), S.end());
    for (int v : S) {
        n.order.push_back(v);
        n.uord.push_back(v);
    }
    n.chain = std::max(L.chain, R.chain) + (int)S.size();
    n.depth = 1 + std::max(L.depth, R.depth);
    return n;
}

}  // namespace detail

namespace detail {

// the plan of one factorisation order (natural panels in order `order`, update order `uord_nat`): positions,
// the tile-level symbolic factorisation (column j's rows = its own rows below the diagonal merged with those
// of its elimination-tree children, minus j; parent = first row) and the dependent chain
inline Plan finish(int NP, const std::vector<std::vector<int>>& lower, const std::vector<int>& order,
                   const std::vector<int>& uord_nat, int tail, int levels) {
    Plan pl;
    pl.NP = NP;
    pl.tail = tail;
    pl.levels = levels;
    pl.ppos.assign(NP, 0);
    pl.pnat.assign(NP, 0);
    for (int q = 0; q < NP; ++q) {
        pl.ppos[order[q]] = q;
        pl.pnat[q] = order[q];
    }
    pl.uord.resize(NP);
    pl.rank.assign(NP, 0);
    for (int q = 0; q < NP; ++q) {
        pl.uord[q] = pl.ppos[uord_nat[q]];
        pl.rank[pl.uord[q]] = q;
    }
    std::vector<std::vector<int>> arows(NP);
    for (int P = 0; P < NP; ++P)
        for (int Q : lower[P]) {
            const int i = std::max(pl.ppos[P], pl.ppos[Q]), j = std::min(pl.ppos[P], pl.ppos[Q]);
            if (i != j) arows[j].push_back(i);
        }
    pl.colrows.assign(NP, {});
    std::vector<std::vector<int>> children(NP);
    for (int j = 0; j < NP; ++j) {
        std::vector<int> r = arows[j];
        for (int c : children[j])
            for (int i : pl.colrows[c])
                if (i != j) r.push_back(i);
        std::sort(r.begin(), r.end());
        r.erase(std::unique(r.begin(), r.end()), r.end());
        pl.colrows[j] = r;
        if (!r.empty()) children[r.front()].push_back(j);
    }
    std::vector<std::vector<int>> rowcols(NP);
    for (int j = 0; j < NP; ++j)
        for (int i : pl.colrows[j]) rowcols[i].push_back(j);
    pl.rowptr.assign(NP + 1, 0);
    for (int i = 0; i < NP; ++i) {
        rowcols[i].push_back(i);   // (columns ascending: j < i were pushed in increasing j)
        pl.rowptr[i + 1] = pl.rowptr[i] + (int)rowcols[i].size();
    }
    pl.cols.reserve(pl.rowptr[NP]);
    for (int i = 0; i < NP; ++i) pl.cols.insert(pl.cols.end(), rowcols[i].begin(), rowcols[i].end());
    // the dependent chain: longest path through the columns (j -> its parent), in panels
    std::vector<int> depth(NP, 1);
    int chain = 0;
    for (int j = 0; j < NP; ++j) {
        chain = std::max(chain, depth[j]);
        if (!pl.colrows[j].empty()) {
            const int par = pl.colrows[j].front();
            depth[par] = std::max(depth[par], depth[j] + 1);
        }
    }
    pl.chain = chain;
    return pl;
}

}  // namespace detail

// NP panels in natural order; the first NPk hold keyframe rows (the rest: free extrinsics, dense rows);
// lower[P]: the natural panels Q <= P whose tile (P, Q) of the system is structurally non-zero.
// levels <= 0: no dissection (natural order); 1: one level (plus the tail); more: nested.  Two orders
// are planned, the interval dissection of the time order (with a loop-closure tail) and the graph
// dissection (level structures; any revisit pattern), and the one with the shorter dependent chain (then
// fewer tiles) is kept; method: 0 both, 1 interval only, 2 graph only.
inline Plan make_plan(int NP, int NPk, const std::vector<std::vector<int>>& lower, int max_levels, bool tail_search,
                      int leaf = 16, int method = 0) {
    // the natural envelope: first coupled panel per row
    std::vector<int> pfirst(NP);
    for (int P = 0; P < NP; ++P) {
        int f = P;
        for (int Q : lower[P]) f = std::min(f, Q);
        pfirst[P] = f;
    }
    Plan best;
    bool have = false;
    auto consider = [&](Plan&& pl) {
        if (!have || pl.chain < best.chain || (pl.chain == best.chain && pl.ntile() < best.ntile())) {
            best = std::move(pl);
            have = true;
        }
    };
    if (method != 2 || max_levels <= 0) {
        // loop-closure tail [c, NPk): the shortest tail after which a one-level cut [A | S1 | B] of [0, c)
        // exists with the shortest chain max(A, B) + S1 + tail (a tail row may reach back anywhere)
        int c_best = NPk;
        if (tail_search && max_levels > 0) {
            // for a cut at a, B = [b, c) is the longest top range of [0, c) whose rows all start at >= a:
            // b = 1 + the last row r < c with pfirst[r] < a (or a), i.e. a running max over pfirst values
            // (mv[v]: the last row below c starting at v), O(NP) per c instead of a scan per (c, a)
            int bestlen = NP + 1;
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
            if (bestlen > NPk) c_best = NPk;   // no cut at all: natural order
        }
        for (int mirror = 0; mirror < (max_levels > 0 ? 2 : 1); ++mirror) {   // (right parts ascending / from the far end)
            detail::Node root = max_levels > 0 ? detail::dissect(0, c_best, lower, leaf, max_levels, mirror != 0)
                                               : detail::dissect(0, c_best, lower, c_best + 1, 0);
            std::vector<int> order = root.order, uord_nat = root.uord;
            for (int P = c_best; P < NP; ++P) {   // the tail, then the extrinsic panels
                order.push_back(P);
                uord_nat.push_back(P);
            }
            consider(detail::finish(NP, lower, order, uord_nat, NPk - c_best, root.depth));
        }
    }
    if (method != 1 && max_levels > 0 && NPk > leaf) {
        std::vector<std::vector<int>> adj(NPk);
        for (int P = 0; P < NPk; ++P)
            for (int Q : lower[P])
                if (Q != P && Q < NPk) { adj[P].push_back(Q); adj[Q].push_back(P); }
        std::vector<int> vs(NPk), mark(NPk, 0);
        for (int P = 0; P < NPk; ++P) vs[P] = P;
        int stamp = 0;
        detail::Node root = detail::dissect_graph(vs, adj, mark, stamp, leaf, max_levels);
        std::vector<int> order = root.order, uord_nat = root.uord;
        for (int P = NPk; P < NP; ++P) {   // the extrinsic panels
            order.push_back(P);
            uord_nat.push_back(P);
        }
        consider(detail::finish(NP, lower, order, uord_nat, 0, root.depth));
    }
    return best;
}

// The distributed factorisation of a partitioned problem (global BA over N GPUs): the
// elimination tree of a plan cut into nranks disjoint subtrees of about equal work, each factored by one rank
// alone, and the top columns above them (the separators the subtrees meet in), factored by every rank once the
// subtrees' contributions are summed.  Columns of different subtrees never share a tile (coupled columns are
// ancestor and descendant), so a landmark's columns lie in one subtree plus the top.  Greedy: from the roots,
// repeatedly split the heaviest subtree of the frontier (its root column moves to the top), and keep the
// frontier with the lowest makespan max(rank load) + top work under a largest-first assignment of its
// subtrees to the ranks.  Returns own[j] (rank of column j's subtree, -1 for the top); deterministic, so
// every rank derives the same split.
inline std::vector<int> split_subtrees(const Plan& pl, int nranks) {
    const int NP = pl.NP;
    std::vector<int> own(NP, -1);
    if (nranks <= 1 || NP == 0) {
        std::fill(own.begin(), own.end(), nranks == 1 ? 0 : -1);
        return own;
    }
    std::vector<int> parent(NP, -1);
    std::vector<std::vector<int>> kids(NP);
    std::vector<double> w(NP), sub(NP);
    for (int j = 0; j < NP; ++j) {
        const double m = (double)pl.colrows[j].size();
        w[j] = 1.0 / 3.0 + 2.0 * m + m * (m - 1.0);   // column j's factor work in 32^3 units
        if (!pl.colrows[j].empty()) {
            parent[j] = pl.colrows[j].front();
            kids[parent[j]].push_back(j);
        }
    }
    for (int j = 0; j < NP; ++j) sub[j] = w[j];
    for (int j = 0; j < NP; ++j)   // (children precede parents: parent > child)
        if (parent[j] >= 0) sub[parent[j]] += sub[j];
    std::vector<int> front;
    for (int j = 0; j < NP; ++j)
        if (parent[j] < 0) front.push_back(j);
    double top = 0.0;
    // largest-first assignment of the frontier subtrees to the ranks: makespan and the owners
    auto assign = [&](const std::vector<int>& fr, std::vector<int>* who) {
        std::vector<int> ord(fr);
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return sub[a] > sub[b] || (sub[a] == sub[b] && a < b); });
        std::vector<double> load(nranks, 0.0);
        if (who) who->assign(NP, -1);
        for (int r : ord) {
            const int k = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            load[k] += sub[r];
            if (who) (*who)[r] = k;
        }
        return *std::max_element(load.begin(), load.end());
    };
    // walk the splits (heaviest frontier subtree first) down to the leaves and keep the cheapest state
    double best = assign(front, nullptr) + top;
    std::vector<int> best_front = front;
    for (int it = 0; it < NP && !front.empty(); ++it) {
        int h = -1;
        for (int r : front)
            if (h < 0 || sub[r] > sub[h] || (sub[r] == sub[h] && r < h)) h = r;
        std::vector<int> fr2;
        for (int r : front)
            if (r != h) fr2.push_back(r);
        for (int c : kids[h]) fr2.push_back(c);
        front.swap(fr2);
        top += w[h];
        if (front.empty()) break;
        const double cost = assign(front, nullptr) + top;
        if (cost < best) {
            best = cost;
            best_front = front;
        }
    }
    front = best_front;
    std::vector<int> who;
    assign(front, &who);
    // every column below a frontier root belongs to that root's rank; the rest is the top
    std::vector<char> is_root(NP, 0);
    for (int r : front) is_root[r] = 1;
    for (int j = NP - 1; j >= 0; --j) {   // parents before children
        if (is_root[j]) own[j] = who[j];
        else if (parent[j] >= 0 && own[parent[j]] >= 0) own[j] = own[parent[j]];
    }
    return own;
}

}  // namespace lba_plan
