// shard_plan.cpp — graph partition and per-shard local graphs.
//
// the network is split into contiguous peer ranges, one per
// shard (GPU), balanced by Σ(row nnz · joined topics).  A shard's local graph
// holds
//   * its owned peers' rows in full, and
//   * one "ghost" row per remote neighbour, holding only that neighbour's
//     connections into the owned range,
// with local peer ids sorted by global id (ghosts below the range, the owned
// range, ghosts above it).  The local CSR is symmetric, so the engine loads it
// as any graph, and record order puts every record an owned
// observer keeps about a ghost into the ghost's row: all state an owned
// observer reads or writes is local.  A directed cross edge (o -> g) exists in
// both shards: in o's shard as an owned-row edge, in g's shard as a ghost-row
// edge.  Listed in (o, g) order the two sides enumerate the same edges in the
// same order, so an exchange needs no index maps: the owned side gathers its
// cross edges to shard S in edge order ("cross-out list"), the other side's
// ghost rows of S's peers are one contiguous block of its local edges.
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "gsim.h"
#include "shard_layout.h"

namespace gsim {

int shard_of_peer(const std::vector<int64_t>& bounds, int64_t g)
{
    return (int)(std::upper_bound(bounds.begin(), bounds.end(), g) - bounds.begin()) - 1;
}

int build_layout(int64_t n, const uint32_t* row_ptr, const uint32_t* col, const int64_t* bounds, int32_t K,
                 int32_t k, ShardLayout* L, std::string* err)
{
    if (K < 1 || K > GSIM_MAX_SHARDS || k < 0 || k >= K) { *err = "shard index out of range"; return GSIM_EINVAL; }
    if (!row_ptr || !col || !bounds || n <= 0) { *err = "empty graph"; return GSIM_EINVAL; }
    if (bounds[0] != 0 || bounds[K] != n) { *err = "bounds must start at 0 and end at n"; return GSIM_EINVAL; }
    for (int s = 0; s < K; ++s)
        if (bounds[s + 1] <= bounds[s]) { *err = "every shard needs at least one peer"; return GSIM_EINVAL; }
    L->k = k;
    L->K = K;
    L->N = n;
    L->E = row_ptr[n];
    L->bounds.assign(bounds, bounds + K + 1);
    const int64_t lo = bounds[k], hi = bounds[k + 1];

    // ghosts: neighbours of owned peers outside the owned range
    std::vector<uint8_t> mark((size_t)n, 0);
    for (int64_t i = lo; i < hi; ++i)
        for (uint32_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
            const uint32_t c = col[e];
            if (c < lo || c >= hi) mark[c] = 1;
        }
    L->gid.clear();
    for (int64_t i = 0; i < lo; ++i)
        if (mark[(size_t)i]) L->gid.push_back((uint32_t)i);
    L->own_lo = (int64_t)L->gid.size();
    for (int64_t i = lo; i < hi; ++i) L->gid.push_back((uint32_t)i);
    L->own_hi = (int64_t)L->gid.size();
    for (int64_t i = hi; i < n; ++i)
        if (mark[(size_t)i]) L->gid.push_back((uint32_t)i);
    L->n_loc = (int64_t)L->gid.size();
    std::vector<int32_t> g2l((size_t)n, -1);
    for (int64_t l = 0; l < L->n_loc; ++l) g2l[L->gid[(size_t)l]] = (int32_t)l;

    // local rows: owned rows in full, ghost rows restricted to the owned range
    L->row_ptr.assign((size_t)L->n_loc + 1, 0);
    L->col.clear();
    L->gidx.clear();
    for (int64_t l = 0; l < L->n_loc; ++l) {
        const uint32_t g = L->gid[(size_t)l];
        uint32_t b = row_ptr[g], en = row_ptr[g + 1];
        if (l < L->own_lo || l >= L->own_hi) {
            b = (uint32_t)(std::lower_bound(col + b, col + en, (uint32_t)lo) - col);
            en = (uint32_t)(std::lower_bound(col + b, col + en, (uint32_t)hi) - col);
        }
        for (uint32_t e = b; e < en; ++e) {
            const int32_t c = g2l[col[e]];
            L->col.push_back((uint32_t)c);
            L->gidx.push_back(e);
        }
        L->row_ptr[(size_t)l + 1] = (uint32_t)L->col.size();
    }
    L->e_loc = (int64_t)L->col.size();
    L->own_e_lo = L->row_ptr[(size_t)L->own_lo];
    L->own_e_hi = L->row_ptr[(size_t)L->own_hi];

    // per shard: its peers' local id range, ghost block and cross-out list
    L->lpeer.assign((size_t)K + 1, 0);
    for (int s = 0; s <= K; ++s)
        L->lpeer[(size_t)s] = (int64_t)(std::lower_bound(L->gid.begin(), L->gid.end(), (uint32_t)std::min<int64_t>(bounds[s], 0xFFFFFFFFll)) - L->gid.begin());
    L->lpeer[(size_t)K] = L->n_loc;
    L->gbase.assign((size_t)K, 0);
    L->gcnt.assign((size_t)K, 0);
    for (int s = 0; s < K; ++s) {
        if (s == k) continue;
        L->gbase[(size_t)s] = L->row_ptr[(size_t)L->lpeer[(size_t)s]];
        L->gcnt[(size_t)s] = (int64_t)L->row_ptr[(size_t)L->lpeer[(size_t)s + 1]] - L->gbase[(size_t)s];
    }
    L->crossout.assign((size_t)K, {});
    L->xq.assign((size_t)L->e_loc, 0xFFFFFFFFu);
    L->n_cross = 0;
    for (int64_t l = L->own_lo; l < L->own_hi; ++l)
        for (uint32_t e = L->row_ptr[(size_t)l]; e < L->row_ptr[(size_t)l + 1]; ++e) {
            const uint32_t c = L->col[e];
            if (c >= L->own_lo && c < L->own_hi) continue;
            const int s = shard_of_peer(L->bounds, L->gid[c]);
            L->xq[e] = (uint32_t)L->crossout[(size_t)s].size();
            L->crossout[(size_t)s].push_back(e);
            ++L->n_cross;
        }
    return GSIM_OK;
}

}  // namespace gsim

using namespace gsim;

extern "C" {

int gsim_shard_partition(int64_t n, const uint32_t* row_ptr, const uint64_t* sub, int32_t shards, int64_t* bounds)
{
    if (n <= 0 || !row_ptr || !bounds || shards < 1 || shards > GSIM_MAX_SHARDS) return GSIM_EINVAL;
    if (n < 64 * (int64_t)shards) return GSIM_ERANGE;    // ranges are whole 64-peer words
    // weight of a peer, per joined topic: its records (row length), a lane
    // group's worth of heartbeat per observer (16 positions), and for a hub
    // row the block-wide selections and PX lists that grow with its length
    // (d^2 / 512: c5's Chung-Lu hubs, all in the lowest ids, made shard 0 the
    // slowest at K = 8 under the records alone)
    std::vector<double> cum((size_t)n + 1, 0.0);
    for (int64_t i = 0; i < n; ++i) {
        const double d = (double)(row_ptr[i + 1] - row_ptr[i]);
        const double s = sub ? (double)__builtin_popcountll(sub[i]) : 1.0;
        const double hub = d > 64.0 ? d * d / 512.0 : 0.0;
        cum[(size_t)i + 1] = cum[(size_t)i] + std::max(1.0, s) * (d + 16.0 + hub) + 1.0;
    }
    bounds[0] = 0;
    for (int32_t s = 1; s < shards; ++s) {
        const double target = cum[(size_t)n] * (double)s / (double)shards;
        int64_t c = (int64_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        c = ((c + 32) / 64) * 64;                          // nearest multiple of 64
        c = std::max<int64_t>(c, bounds[s - 1] + 64);
        c = std::min<int64_t>(c, n - 64 * (int64_t)(shards - s));
        bounds[s] = c;
    }
    bounds[shards] = n;
    return GSIM_OK;
}

int gsim_shard_layout_info(int64_t n, const uint32_t* row_ptr, const uint32_t* col, const int64_t* bounds,
                           int32_t shards, int32_t shard, gsim_shard_info* out)
{
    if (!out) return GSIM_EINVAL;
    ShardLayout L;
    std::string err;
    int rc = build_layout(n, row_ptr, col, bounds, shards, shard, &L, &err);
    if (rc) return rc;
    out->shard = shard;
    out->shards = shards;
    out->n_local = L.n_loc;
    out->e_local = L.e_loc;
    out->own_lo = L.own_lo;
    out->own_hi = L.own_hi;
    out->own_e_lo = L.own_e_lo;
    out->own_e_hi = L.own_e_hi;
    out->n_cross = L.n_cross;
    return GSIM_OK;
}

int gsim_shard_layout(int64_t n, const uint32_t* row_ptr, const uint32_t* col, const int64_t* bounds,
                      int32_t shards, int32_t shard, uint32_t* gid, uint32_t* row_ptr_l, uint32_t* col_l,
                      uint64_t* gidx, int64_t* ghost_base, int64_t* ghost_count, uint32_t* cross_out,
                      int64_t* cross_count)
{
    ShardLayout L;
    std::string err;
    int rc = build_layout(n, row_ptr, col, bounds, shards, shard, &L, &err);
    if (rc) return rc;
    if (gid) std::copy(L.gid.begin(), L.gid.end(), gid);
    if (row_ptr_l) std::copy(L.row_ptr.begin(), L.row_ptr.end(), row_ptr_l);
    if (col_l) std::copy(L.col.begin(), L.col.end(), col_l);
    if (gidx) std::copy(L.gidx.begin(), L.gidx.end(), gidx);
    int64_t off = 0;
    for (int s = 0; s < shards; ++s) {
        if (ghost_base) ghost_base[s] = L.gbase[(size_t)s];
        if (ghost_count) ghost_count[s] = L.gcnt[(size_t)s];
        if (cross_count) cross_count[s] = (int64_t)L.crossout[(size_t)s].size();
        if (cross_out) std::copy(L.crossout[(size_t)s].begin(), L.crossout[(size_t)s].end(), cross_out + off);
        off += (int64_t)L.crossout[(size_t)s].size();
    }
    return GSIM_OK;
}

}  // extern "C"
