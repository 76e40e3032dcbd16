// graphgen.cpp — synthetic peer graphs (SURVEY.md §8(d) inputs).
//
// The reference tests wire hosts with connect/sparseConnect/denseConnect
// (floodsub_test.go:58-100); the simulated networks here are seeded random
// k-regular graphs built by the configuration model: stubs are shuffled and
// paired, then self-loops and multi-edges are repaired by random double-edge
// swaps until the graph is simple.
#include <algorithm>
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
