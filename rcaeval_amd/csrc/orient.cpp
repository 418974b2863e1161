// orient.cpp — host orientation of the PC skeleton (no device work).
//
// Restates causal-learn 0.1.3.3 [U] (not on disk; pinned requirements.txt:20):
//   pc_alg: cg_2 = UCSepset.uc_sepset(cg_1, uc_priority); cg = Meek.meek(cg_2)
// over the enumerations of the vendored lib/causallearn/graph/GraphClass.py:
//   find_tails / find_arrow_heads :108-116 (np.where row-major, entries (col, row))
//   find_adj :145-147 (tails + arrow heads)
//   find_unshielded_triples :157-165, find_triangles :167-176, find_kites :178-188
//   (itertools.permutations order), and GeneralGraph [U] edge semantics:
//   add_edge(Edge(i, j, TAIL, ARROW)) is a no-op on an existing non-bidirected edge, else
//   g[i,j] = -1, g[j,i] = 1 and adjust_dpath(i, j); remove_edge of a fully directed edge
//   calls reconstitute_dpath(get_graph_edges()); is_ancestor_of(a, b) = dpath[b, a] == 1.
// uc_sepset(priority=2): for (x, y, z) in unshielded triples with x < z, if y is in no S of
// sepset[x, z] (= the union of both sides' unions at the removal depth) and neither y->x nor
// y->z is fully directed: re-orient x->y and z->y. Meek: R1 over triples, R2 over
// triangles, R3 over kites until no change, skipping an orientation that would point at
// an ancestor (is_ancestor_of check). Parity of these [U] details is unpinned offline.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "pcgpu.h"

namespace {

struct Graph {
    int64_t n;
    std::vector<int8_t> g;      // endpoint codes
    std::vector<uint8_t> dpath; // dpath[j * n + i] == 1 <=> i is an ancestor of j

    int8_t &at(int64_t i, int64_t j) { return g[i * n + j]; }
    int8_t at(int64_t i, int64_t j) const { return g[i * n + j]; }

    void adjust_dpath(int64_t i, int64_t j) {
        uint8_t *dp = dpath.data();
        dp[j * n + i] = 1;
        for (int64_t k = 0; k < n; ++k) {
            if (dp[i * n + k] == 1) dp[j * n + k] = 1;
            if (dp[k * n + j] == 1) dp[k * n + i] = 1;
        }
    }
    void reconstitute_dpath() {
        for (int64_t i = 0; i < n; ++i) adjust_dpath(i, i);
        // get_graph_edges(): i ascending, j > i ascending; Edge normalised tail-first for
        // directed edges; edges.pop() consumes from the end.
        std::vector<std::pair<int64_t, int64_t>> edges;
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = i + 1; j < n; ++j) {
                const int8_t e1 = at(i, j), e2 = at(j, i);
                if (e1 == 0 && e2 == 0) continue;
                if (e1 == 1 && e2 == -1) edges.push_back({j, i});  // i <- j: node1 = j
                else edges.push_back({i, j});
            }
        while (!edges.empty()) {
            auto e = edges.back();
            edges.pop_back();
            adjust_dpath(e.first, e.second);
        }
    }
    bool is_fully_directed(int64_t i, int64_t j) const { return at(i, j) == -1 && at(j, i) == 1; }
    bool is_undirected(int64_t i, int64_t j) const { return at(i, j) == -1 && at(j, i) == -1; }
    bool is_ancestor_of(int64_t a, int64_t b) const { return dpath[b * n + a] == 1; }
    bool adjacent(int64_t i, int64_t j) const { return at(i, j) != 0; }

    // remove the edge between i and j (GeneralGraph.remove_edge(get_edge(i, j)))
    void remove_edge(int64_t i, int64_t j) {
        const bool directed = is_fully_directed(i, j) || is_fully_directed(j, i);
        at(i, j) = 0;
        at(j, i) = 0;
        if (directed) reconstitute_dpath();
    }
    // add_edge(Edge(i, j, TAIL, ARROW))
    void add_directed(int64_t i, int64_t j) {
        const int8_t e1 = at(i, j), e2 = at(j, i);
        const bool bidirected = e1 == 1 && e2 == 1;
        const bool existing = !bidirected && (e1 != 0 || e2 != 0);
        if (existing) return;
        if (bidirected) return;  // not produced by PC orientation
        at(j, i) = 1;
        at(i, j) = -1;
        adjust_dpath(i, j);
    }
};

// find_adj(): tails then arrow heads, each np.where row-major with entries (col, row)
std::vector<std::pair<int32_t, int32_t>> find_adj(const Graph &G) {
    std::vector<std::pair<int32_t, int32_t>> adj;
    for (int code : {-1, 1})
        for (int64_t r = 0; r < G.n; ++r)
            for (int64_t c = 0; c < G.n; ++c)
                if (G.at(r, c) == code) adj.push_back({(int32_t)c, (int32_t)r});
    return adj;
}

// background knowledge [U] (causal-learn BackgroundKnowledge): directed relations i -> j
struct BK {
    int64_t n = 0;
    const uint8_t *forb = nullptr, *req = nullptr;
    bool forbidden(int64_t i, int64_t j) const { return forb && forb[i * n + j]; }
    bool required(int64_t i, int64_t j) const { return req && req[i * n + j]; }
    bool any() const { return forb || req; }
};

struct Triple { int32_t i, j, k; };
struct Kite { int32_t i, j, k, l; };

// permutations(Adj, 2) filtered: pair0 = (i, j), pair1 = (j', k) with j' == j, i != k
template <class Pred>
std::vector<Triple> enumerate_triples(const Graph &G, const std::vector<std::pair<int32_t, int32_t>> &adj,
                                      Pred keep) {
    // positions of Adj entries by first element, ascending
    std::vector<std::vector<int32_t>> by_first(G.n);
    for (size_t b = 0; b < adj.size(); ++b) by_first[adj[b].first].push_back((int32_t)b);
    std::vector<Triple> out;
    for (size_t a = 0; a < adj.size(); ++a) {
        const int32_t i = adj[a].first, j = adj[a].second;
        for (int32_t b : by_first[j]) {
            if ((size_t)b == a) continue;
            const int32_t k = adj[b].second;
            if (i != k && keep(i, j, k)) out.push_back({i, j, k});
        }
    }
    return out;
}

struct Sepsets {                        // sepset[x, z] membership: both sides' rows, keyed by (min, max)
    int64_t n, W;
    std::unordered_map<uint64_t, std::vector<uint64_t>> rows;
    Sepsets(int64_t n_, const int32_t *sep_xy, const uint64_t *sep_bits, int64_t count) : n(n_), W((n_ + 63) / 64) {
        for (int64_t r = 0; r < count; ++r) {
            const int64_t x = sep_xy[2 * r], y = sep_xy[2 * r + 1];
            auto &row = rows[key(x, y)];
            if (row.empty()) row.assign(W, 0);
            for (int64_t w = 0; w < W; ++w) row[w] |= sep_bits[r * W + w];
        }
    }
    uint64_t key(int64_t a, int64_t b) const { return (uint64_t)std::min(a, b) * (uint64_t)n + (uint64_t)std::max(a, b); }
    bool contains(int64_t x, int64_t z, int64_t y) const {   // y in some S of sepset[x, z]
        auto it = rows.find(key(x, z));
        if (it == rows.end()) return false;
        return ((it->second[y >> 6] >> (y & 63)) & 1ull) != 0;
    }
};

void init_graph(Graph &G, int64_t n, const uint8_t *adj) {
    G.n = n;
    G.g.assign(n * n, 0);
    G.dpath.assign(n * n, 0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j)
            if (i != j && adj[i * n + j]) G.at(i, j) = -1;
    for (int64_t i = 0; i < n; ++i) G.adjust_dpath(i, i);  // GeneralGraph.__init__: reconstitute_dpath([])
}

// uc_sepset's R0 list: unshielded triples (x, y, z), x < z, in find_unshielded_triples order,
// with y in no S of sepset[x, z]. The check does not depend on orientation, so priority 2's
// in-loop test and priority 3/4's R0 filter select the same triples.
std::vector<Triple> uc_candidates(const Graph &G, const Sepsets &sep) {
    const auto A = find_adj(G);
    const auto UT = enumerate_triples(G, A, [&](int32_t i, int32_t, int32_t k) { return G.at(i, k) == 0; });
    std::vector<Triple> R0;
    for (const Triple &t : UT)
        if (t.i < t.k && !sep.contains(t.i, t.k, t.j)) R0.push_back(t);
    return R0;
}

// orient_by_background_knowledge [U] (pc_alg, before uc_sepset): every undirected edge in
// get_graph_edges order (node1 < node2): node1 -> node2 if node2 -> node1 is forbidden, else
// node2 -> node1 if node1 -> node2 is forbidden, else the required direction
void orient_by_bk(Graph &G, const BK &bk) {
    for (int64_t i = 0; i < G.n; ++i)
        for (int64_t j = i + 1; j < G.n; ++j) {
            if (!G.is_undirected(i, j)) continue;
            int64_t a = -1, b = -1;
            if (bk.forbidden(j, i)) a = i, b = j;
            else if (bk.forbidden(i, j)) a = j, b = i;
            else if (bk.required(j, i)) a = j, b = i;
            else if (bk.required(i, j)) a = i, b = j;
            if (a < 0) continue;
            G.remove_edge(i, j);
            G.add_directed(a, b);
        }
}

// uc_sepset's background-knowledge skip [U]: x->y or z->y forbidden, y->x or y->z required
bool bk_blocks_collider(const BK &bk, int64_t x, int64_t y, int64_t z) {
    return bk.forbidden(x, y) || bk.forbidden(z, y) || bk.required(y, x) || bk.required(y, z);
}
// Meek's skip [U]: orienting i->j is forbidden, or j->i is required
bool bk_blocks(const BK &bk, int64_t i, int64_t j) { return bk.forbidden(i, j) || bk.required(j, i); }

// the collider step shared by priorities 2, 3 and 4: x->y<-z unless y->x or y->z is fully directed
void apply_colliders(Graph &G, const Triple *T, int64_t count, const BK &bk = BK()) {
    for (int64_t q = 0; q < count; ++q) {
        const int64_t x = T[q].i, y = T[q].j, z = T[q].k;
        if (bk.any() && bk_blocks_collider(bk, x, y, z)) continue;
        if (!G.is_fully_directed(y, x) && !G.is_fully_directed(y, z)) {
            if (G.adjacent(x, y)) G.remove_edge(x, y);
            G.add_directed(x, y);
            if (G.adjacent(z, y)) G.remove_edge(z, y);
            G.add_directed(z, y);
        }
    }
}

// Meek.meek [U]: triple / triangle / kite lists computed once from cg_new = deepcopy(cg_2)
void meek(Graph &G, const BK &bk = BK()) {
    const int64_t n = G.n;
    const auto A = find_adj(G);
    const auto UT = enumerate_triples(G, A, [&](int32_t i, int32_t, int32_t k) { return G.at(i, k) == 0; });
    // (i, k) in Adj  <=>  g[k, i] in {-1, 1}
    const auto Tri = enumerate_triples(G, A, [&](int32_t i, int32_t, int32_t k) {
        const int8_t v = G.at(k, i);
        return v == -1 || v == 1;
    });
    // kites from permutations(Tri, 2)
    std::vector<Kite> Kites;
    {
        std::unordered_map<uint64_t, std::vector<int32_t>> by_ik;
        for (size_t b = 0; b < Tri.size(); ++b)
            by_ik[(uint64_t)Tri[b].i * (uint64_t)n + (uint64_t)Tri[b].k].push_back((int32_t)b);
        for (size_t a = 0; a < Tri.size(); ++a) {
            const Triple &p0 = Tri[a];
            auto it = by_ik.find((uint64_t)p0.i * (uint64_t)n + (uint64_t)p0.k);
            for (int32_t b : it->second) {
                if ((size_t)b == a) continue;
                const Triple &p1 = Tri[b];
                if (p0.j < p1.j && G.at(p0.j, p1.j) == 0) Kites.push_back({p0.i, p0.j, p1.j, p0.k});
            }
        }
    }
    bool loop = true;
    while (loop) {
        loop = false;
        for (const Triple &t : UT) {  // R1
            const int64_t i = t.i, j = t.j, k = t.k;
            if (G.is_fully_directed(i, j) && G.is_undirected(j, k)) {
                if (!G.adjacent(j, k)) continue;
                if (bk.any() && bk_blocks(bk, j, k)) continue;
                if (G.is_ancestor_of(k, j)) continue;
                G.remove_edge(j, k);
                G.add_directed(j, k);
                loop = true;
            }
        }
        for (const Triple &t : Tri) {  // R2
            const int64_t i = t.i, j = t.j, k = t.k;
            if (G.is_fully_directed(i, j) && G.is_fully_directed(j, k) && G.is_undirected(i, k)) {
                if (!G.adjacent(i, k)) continue;
                if (bk.any() && bk_blocks(bk, i, k)) continue;
                if (G.is_ancestor_of(k, i)) continue;
                G.remove_edge(i, k);
                G.add_directed(i, k);
                loop = true;
            }
        }
        for (const Kite &q : Kites) {  // R3
            const int64_t i = q.i, j = q.j, k = q.k, l = q.l;
            if (G.is_undirected(i, j) && G.is_undirected(i, k) && G.is_fully_directed(j, l) &&
                G.is_fully_directed(k, l) && G.is_undirected(i, l)) {
                if (!G.adjacent(i, l)) continue;
                if (bk.any() && bk_blocks(bk, i, l)) continue;
                if (G.is_ancestor_of(l, i)) continue;
                G.remove_edge(i, l);
                G.add_directed(i, l);
                loop = true;
            }
        }
    }
}

}  // namespace

extern "C" int pcg_orient(int64_t n, const uint8_t *adj, const int32_t *sep_xy, const uint64_t *sep_bits,
                          int64_t count, int priority, int32_t *graph) {
    if (n < 1 || !adj || !graph || (count > 0 && (!sep_xy || !sep_bits))) return PCG_ERR_INVALID;
    if (priority != 2) return PCG_ERR_INVALID;  // 3/4 need CI tests: pcg_uc_candidates + pcg_orient_triples
    Graph G;
    init_graph(G, n, adj);
    const Sepsets sep(n, sep_xy, sep_bits, count);
    const auto R0 = uc_candidates(G, sep);      // uc_sepset(priority = 2) on cg_new = deepcopy(cg)
    apply_colliders(G, R0.data(), (int64_t)R0.size());
    meek(G);
    for (int64_t i = 0; i < n * n; ++i) graph[i] = G.g[i];
    return PCG_OK;
}

extern "C" int pcg_uc_candidates(int64_t n, const uint8_t *adj, const int32_t *sep_xy, const uint64_t *sep_bits,
                                 int64_t count, int32_t *triples, int64_t capacity, int64_t *total) {
    if (n < 1 || !adj || !total || (count > 0 && (!sep_xy || !sep_bits)) || (capacity > 0 && !triples))
        return PCG_ERR_INVALID;
    Graph G;
    init_graph(G, n, adj);
    const auto R0 = uc_candidates(G, Sepsets(n, sep_xy, sep_bits, count));
    *total = (int64_t)R0.size();
    const int64_t m = std::min<int64_t>(capacity, (int64_t)R0.size());
    for (int64_t q = 0; q < m; ++q) {
        triples[3 * q] = R0[q].i;
        triples[3 * q + 1] = R0[q].j;
        triples[3 * q + 2] = R0[q].k;
    }
    return PCG_OK;
}

extern "C" int pcg_orient_triples(int64_t n, const uint8_t *adj, const int32_t *triples, int64_t tcount,
                                  int32_t *graph) {
    if (n < 1 || !adj || !graph || tcount < 0 || (tcount > 0 && !triples)) return PCG_ERR_INVALID;
    std::vector<Triple> T((size_t)tcount);
    for (int64_t q = 0; q < tcount; ++q) {
        T[q] = {triples[3 * q], triples[3 * q + 1], triples[3 * q + 2]};
        if (T[q].i < 0 || T[q].j < 0 || T[q].k < 0 || T[q].i >= n || T[q].j >= n || T[q].k >= n)
            return PCG_ERR_INVALID;
    }
    Graph G;
    init_graph(G, n, adj);
    apply_colliders(G, T.data(), tcount);
    meek(G);
    for (int64_t i = 0; i < n * n; ++i) graph[i] = G.g[i];
    return PCG_OK;
}

extern "C" int pcg_orient_bk(int64_t n, const uint8_t *adj, const int32_t *sep_xy, const uint64_t *sep_bits,
                             int64_t count, int priority, const int32_t *triples, const double *scores,
                             int64_t tcount, const uint8_t *forbidden, const uint8_t *required, int32_t *graph) {
    if (n < 1 || !adj || !graph || (count > 0 && (!sep_xy || !sep_bits))) return PCG_ERR_INVALID;
    if (priority != 2 && priority != 3 && priority != 4) return PCG_ERR_INVALID;
    if (priority != 2 && (tcount < 0 || (tcount > 0 && (!triples || !scores)))) return PCG_ERR_INVALID;
    BK bk;
    bk.n = n;
    bk.forb = forbidden;
    bk.req = required;
    Graph G;
    init_graph(G, n, adj);
    orient_by_bk(G, bk);
    // uc_sepset works on its deepcopy of the oriented graph: R0 in that graph's
    // find_unshielded_triples order (the set is the skeleton's, the order is not)
    std::vector<Triple> R0 = uc_candidates(G, Sepsets(n, sep_xy, sep_bits, count));
    if (priority != 2) {
        // priorities 3 / 4: the caller scored the candidates (any order); stable sort by score,
        // ascending (3) or descending (4), ties in R0 order (sort_dict_ascending)
        std::unordered_map<uint64_t, double> score;
        score.reserve((size_t)tcount * 2);
        auto key = [n](int64_t i, int64_t j, int64_t k) { return ((uint64_t)i * n + j) * n + k; };
        for (int64_t q = 0; q < tcount; ++q) {
            const int64_t i = triples[3 * q], j = triples[3 * q + 1], k = triples[3 * q + 2];
            if (i < 0 || j < 0 || k < 0 || i >= n || j >= n || k >= n) return PCG_ERR_INVALID;
            score[key(i, j, k)] = scores[q];
        }
        std::vector<std::pair<double, Triple>> sc;
        sc.reserve(R0.size());
        for (const Triple &t : R0) {
            auto it = score.find(key(t.i, t.j, t.k));
            if (it == score.end()) return PCG_ERR_INVALID;
            sc.push_back({it->second, t});
        }
        if (priority == 3)
            std::stable_sort(sc.begin(), sc.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        else
            std::stable_sort(sc.begin(), sc.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
        for (size_t q = 0; q < sc.size(); ++q) R0[q] = sc[q].second;
    }
    apply_colliders(G, R0.data(), (int64_t)R0.size(), bk);
    meek(G, bk);
    for (int64_t i = 0; i < n * n; ++i) graph[i] = G.g[i];
    return PCG_OK;
}
