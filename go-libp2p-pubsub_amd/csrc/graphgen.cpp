// graphgen.cpp — synthetic peer graphs (SURVEY.md §8(d) inputs).
//
// The reference tests wire hosts with connect/sparseConnect/denseConnect
// (floodsub_test.go:58-100); the simulated networks here are seeded random
// k-regular graphs built by the configuration model: stubs are shuffled and
// paired, then self-loops and multi-edges are repaired by random double-edge
// swaps until the graph is simple.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "gsim.h"

namespace {

struct SplitMix64 {
    uint64_t s;
    uint64_t next()
    {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t n) { return next() % n; }
};

inline uint64_t ekey(uint32_t a, uint32_t b)
{
    if (a > b) std::swap(a, b);
    return ((uint64_t)a << 32) | b;
}

}  // namespace

extern "C" int gsim_gen_random_regular(int64_t n, int32_t k, uint64_t seed, uint32_t* row_ptr, uint32_t* col,
                                       uint8_t* outbound)
{
    if (n <= 1 || k <= 0 || k >= n || ((n * (int64_t)k) & 1) || !row_ptr || !col) return GSIM_EINVAL;
    if (n * (int64_t)k >= (int64_t)UINT32_MAX) return GSIM_ERANGE;
    const int64_t m = n * (int64_t)k / 2;
    SplitMix64 rng{seed};
    std::vector<uint32_t> stubs((size_t)(n * k));
    for (int64_t i = 0; i < n; ++i)
        for (int32_t q = 0; q < k; ++q) stubs[(size_t)(i * k + q)] = (uint32_t)i;
    for (int64_t i = (int64_t)stubs.size() - 1; i > 0; --i) std::swap(stubs[(size_t)i], stubs[rng.below((uint64_t)i + 1)]);
    std::vector<uint32_t> ea((size_t)m), eb((size_t)m);
    for (int64_t e = 0; e < m; ++e) { ea[(size_t)e] = stubs[(size_t)(2 * e)]; eb[(size_t)e] = stubs[(size_t)(2 * e + 1)]; }
    stubs.clear();
    stubs.shrink_to_fit();

    std::vector<uint64_t> keyidx((size_t)m);
    std::vector<int64_t> bad;
    for (int pass = 0; pass < 1000; ++pass) {
        // find self loops and duplicates (all but the first copy of a key)
        for (int64_t e = 0; e < m; ++e) keyidx[(size_t)e] = (uint64_t)e;
        std::vector<uint64_t> keys((size_t)m);
        for (int64_t e = 0; e < m; ++e) keys[(size_t)e] = ekey(ea[(size_t)e], eb[(size_t)e]);
        std::sort(keyidx.begin(), keyidx.end(), [&](uint64_t x, uint64_t y) {
            return keys[x] != keys[y] ? keys[x] < keys[y] : x < y;
        });
        bad.clear();
        for (int64_t r = 0; r < m; ++r) {
            const uint64_t e = keyidx[(size_t)r];
            if (ea[e] == eb[e] || (r > 0 && keys[keyidx[(size_t)r - 1]] == keys[e])) bad.push_back((int64_t)e);
        }
        if (bad.empty()) break;
        for (int64_t e : bad) {
            const uint64_t o = rng.below((uint64_t)m);
            if ((int64_t)o == e) continue;
            if (rng.next() & 1) std::swap(ea[o], eb[o]);
            std::swap(eb[(size_t)e], ea[o]);   // (a,b),(c,d) -> (a,c),(b,d)
        }
        if (pass == 999) return GSIM_ERANGE;
    }

    // CSR with both directions; rows sorted
    for (int64_t i = 0; i <= n; ++i) row_ptr[i] = (uint32_t)(i * k);
    std::vector<uint32_t> fill((size_t)n, 0);
    std::vector<uint8_t> ob;
    if (outbound) ob.assign((size_t)(n * k), 0);
    for (int64_t e = 0; e < m; ++e) {
        const uint32_t a = ea[(size_t)e], b = eb[(size_t)e];
        const uint8_t bit = (uint8_t)(rng.next() & 1);   // who initiated
        const uint32_t pa = row_ptr[a] + fill[a]++, pb = row_ptr[b] + fill[b]++;
        col[pa] = b;
        col[pb] = a;
        if (outbound) { ob[pa] = bit; ob[pb] = (uint8_t)(1 - bit); }
    }
    std::vector<std::pair<uint32_t, uint8_t>> tmp((size_t)k);
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t b = row_ptr[i];
        for (int32_t q = 0; q < k; ++q) tmp[(size_t)q] = {col[b + q], outbound ? ob[b + q] : (uint8_t)0};
        std::sort(tmp.begin(), tmp.end());
        for (int32_t q = 0; q < k; ++q) {
            col[b + q] = tmp[(size_t)q].first;
            if (outbound) outbound[b + q] = tmp[(size_t)q].second;
        }
    }
    return GSIM_OK;
}

// Chung-Lu power law: expected degree of peer i
// proportional to (i + i0)^(-1/(exponent-1)), scaled to `mean`, capped at
// max_degree.  m = round(sum w / 2) endpoint pairs are drawn by inverse CDF;
// self loops and repeated pairs are dropped; pairs are then accepted in
// drawing order while both ends are below the cap (the model of
// gsim.graphs.power_law, with its own seeded stream: the same distribution,
// not the same graph).  Outbound: the first endpoint drawn dials.
// Two calls: with col == nullptr only *n_edges (the directed edge count) is
// computed; then row_ptr (n+1), col and outbound (*n_edges each) are filled.
extern "C" int gsim_gen_power_law(int64_t n, double mean, double exponent, int32_t max_degree, double i0,
                                  uint64_t seed, uint32_t* row_ptr, uint32_t* col, uint8_t* outbound,
                                  int64_t* n_edges)
{
    if (n <= 1 || mean <= 0 || exponent <= 2.0 || max_degree <= 0 || i0 < 1.0 || !n_edges) return GSIM_EINVAL;
    if (n >= (int64_t)UINT32_MAX) return GSIM_ERANGE;
    // Vose alias table over the capped weights: O(1) per endpoint drawn
    std::vector<double> w((size_t)n);
    double sum = 0;
    const double ex = -1.0 / (exponent - 1.0);
    for (int64_t i = 0; i < n; ++i) sum += std::pow((double)i + i0, ex);
    const double scale = mean * (double)n / sum;
    double acc = 0;
    for (int64_t i = 0; i < n; ++i) {
        w[(size_t)i] = std::min(std::pow((double)i + i0, ex) * scale, (double)max_degree);
        acc += w[(size_t)i];
    }
    const int64_t m = (int64_t)std::llround(acc / 2.0);
    std::vector<double> prob((size_t)n);
    std::vector<uint32_t> alias((size_t)n);
    {
        std::vector<uint32_t> small, large;
        for (int64_t i = 0; i < n; ++i) {
            prob[(size_t)i] = w[(size_t)i] * (double)n / acc;
            (prob[(size_t)i] < 1.0 ? small : large).push_back((uint32_t)i);
        }
        while (!small.empty() && !large.empty()) {
            const uint32_t s0 = small.back(), l0 = large.back();
            small.pop_back();
            alias[s0] = l0;
            prob[l0] = (prob[l0] + prob[s0]) - 1.0;
            if (prob[l0] < 1.0) { large.pop_back(); small.push_back(l0); }
        }
        for (uint32_t x : large) prob[x] = 1.0;
        for (uint32_t x : small) prob[x] = 1.0;
    }
    w.clear();
    w.shrink_to_fit();
    SplitMix64 rng{seed};
    auto draw = [&]() -> uint32_t {
        const uint64_t r = rng.next();
        const uint32_t i = (uint32_t)((r >> 32) * (uint64_t)n >> 32);
        const double u = (double)(r & 0xFFFFFFFFull) * (1.0 / 4294967296.0);
        return u < prob[i] ? i : alias[i];
    };
    struct Pair { uint64_t key; uint32_t idx; uint8_t lo_first; };
    std::vector<Pair> pairs;
    pairs.reserve((size_t)m);
    for (int64_t q = 0; q < m; ++q) {
        const uint32_t u = draw(), v = draw();
        if (u == v) continue;
        pairs.push_back(Pair{ekey(u, v), (uint32_t)pairs.size(), (uint8_t)(u < v ? 1 : 0)});
    }
    prob.clear();
    prob.shrink_to_fit();
    alias.clear();
    alias.shrink_to_fit();
    // first occurrence of every pair, then back in drawing order
    std::sort(pairs.begin(), pairs.end(), [](const Pair& x, const Pair& y) {
        return x.key != y.key ? x.key < y.key : x.idx < y.idx;
    });
    size_t nu = 0;
    for (size_t q = 0; q < pairs.size(); ++q)
        if (q == 0 || pairs[q].key != pairs[q - 1].key) pairs[nu++] = pairs[q];
    pairs.resize(nu);
    std::sort(pairs.begin(), pairs.end(), [](const Pair& x, const Pair& y) { return x.idx < y.idx; });
    std::vector<uint8_t> keep(pairs.size(), 1);
    std::vector<uint32_t> deg((size_t)n, 0);
    int64_t E = 0;
    for (size_t q = 0; q < pairs.size(); ++q) {
        const uint32_t a = (uint32_t)(pairs[q].key >> 32), b = (uint32_t)pairs[q].key;
        if (deg[a] >= (uint32_t)max_degree || deg[b] >= (uint32_t)max_degree) { keep[q] = 0; continue; }
        ++deg[a];
        ++deg[b];
        E += 2;
    }
    *n_edges = E;
    if (E >= (int64_t)UINT32_MAX) return GSIM_ERANGE;
    if (!col) return GSIM_OK;
    if (!row_ptr) return GSIM_EINVAL;
    row_ptr[0] = 0;
    for (int64_t i = 0; i < n; ++i) row_ptr[i + 1] = row_ptr[i] + deg[(size_t)i];
    std::vector<uint32_t> fill(row_ptr, row_ptr + n);
    for (size_t q = 0; q < pairs.size(); ++q) {
        if (!keep[q]) continue;
        const uint32_t a = (uint32_t)(pairs[q].key >> 32), b = (uint32_t)pairs[q].key;
        const uint32_t ea = fill[a]++, eb = fill[b]++;
        col[ea] = b;
        col[eb] = a;
        if (outbound) {
            outbound[ea] = pairs[q].lo_first;           // the lower id dialled
            outbound[eb] = (uint8_t)(1 - pairs[q].lo_first);
        }
    }
    // sorted rows (outbound follows its edge)
    std::vector<uint64_t> tmp;
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t b0 = row_ptr[i], b1 = row_ptr[i + 1];
        if (b1 - b0 < 2) continue;
        if (!outbound) { std::sort(col + b0, col + b1); continue; }
        tmp.resize(b1 - b0);
        for (uint32_t e = b0; e < b1; ++e) tmp[e - b0] = ((uint64_t)col[e] << 8) | outbound[e];
        std::sort(tmp.begin(), tmp.end());
        for (uint32_t e = b0; e < b1; ++e) { col[e] = (uint32_t)(tmp[e - b0] >> 8); outbound[e] = (uint8_t)tmp[e - b0]; }
    }
    return GSIM_OK;
}
