// engine.hip — device state, hot-path kernels and the C ABI (include/gsim.h).
//
// The reference keeps one peerScore (score.go:64-86) and one GossipSubRouter
// (gossipsub.go:420-477) per node, each a set of Go maps.  Here the whole
// simulated network is one structure-of-arrays over a CSR peer graph: row i is
// observer i's peerStats map, column j its neighbour, and every per-topic
// topicStats field is a [T][E] topic-major array so that a wavefront walking
// consecutive edges of one topic reads consecutive addresses.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gsim.h"
#include "gsim_internal.h"
#include "philox.h"

using namespace gsim;

std::atomic<unsigned long long> gsim::g_host_syncs{0};

extern "C" int gsim_host_sync_count(uint64_t* out)
{
    if (!out) return GSIM_EINVAL;
    *out = g_host_syncs.load(std::memory_order_relaxed);
    return GSIM_OK;
}

// ---------------------------------------------------------------------------
// Kernel 1:peerScore.refreshScores (score.go:504-565) fused with
// peerScore.score (score.go:265-342).  One thread per record (record order,
// the record of observer col[r] about neighbour owner[r]),
// grid-stride; the topic loop reads the [T][E] arrays at t*E + r, so each
// wave-instruction touches 64 consecutive records of one topic (coalesced),
// and the P5 gather p5[owner[r]] hits one or two rows per wave.
// Topic parameters are wave-uniform (scalar loads).  Operation order is the
// reference's, compiled with -ffp-contract=off: results are bit-identical to
// the CPU oracle.
#ifndef GSIM_REFRESH_GRAFT_EAGER
#define GSIM_REFRESH_GRAFT_EAGER 0
#endif
template <bool REFRESH, bool SCORE>
__global__ __launch_bounds__(256) void k_refresh_score(ScoreArgs a_)
{
    const ScoreArgs& a0 = a_;
    if (a0.gate && *a0.gate == 0) return;
    // every invalidMessageDeliveries counter is zero while the flag is clear:
    // those planes are not read (C3: 4 GB per pass), a zero is what they hold
    const bool inv_on = !a0.inv_live || *a0.inv_live != 0;
    bool inv_left = false;           // a record still holds a non-zero counter after this pass
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a0.E; e += stride) {
        const ScoreArgs& a = kernarg0(a_);   // (re-read per record: SGPR pressure)
        if (a.sharded) {   // a record of a ghost observer belongs to another shard
            const uint32_t o = a.col[e];
            if (o < a.olo || o >= a.ohi) continue;
        }
        const uint8_t st = a.estate[e];
        if (!(st & GSIM_ES_TRACKED)) {
            if (SCORE) a.score[e] = 0.0;
            if (REFRESH && a.pen[e]) a.pen[e] = 0;      // AddPenalty without peerStats: no-op
            continue;
        }
        const bool conn = (st & GSIM_ES_CONNECTED) != 0;
        if (REFRESH && !conn && a.now > a.expire[e]) {
            // retention elapsed: delete(ps.peerStats, p) (score.go:512-516)
            a.estate[e] = 0;
            a.bp[e] = 0.0;
            a.expire[e] = 0;
            a.pen[e] = 0;
            const uint64_t mj = smask_of(a.smask, a.owner[e]);
            for (int32_t t = 0; t < a.T; ++t) {
                if (!slot_has(mj, t)) continue;
                const int64_t i = slot_idx(mj, t, a.E, e);
                a.first[i] = 0.0; a.meshd[i] = 0.0; a.fail[i] = 0.0; a.invalid[i] = 0.0; a.mcnt[i] = 0;
                a.graft[i] = 0; a.mtime[i] = 0; a.tflags[i] = 0;
            }
            *a.purged = 1;
            if (a.p6row) a.p6row[a.col[e]] = 1;        // the observer's tracked set shrank
            if (SCORE) a.score[e] = 0.0;
            continue;
        }
        const bool decay = REFRESH && conn;   // retained scores are not decayed
        // topics the observer joined (the others hold zero records: skipping
        // them leaves every value and the score's sum unchanged)
        // ... and the topics the neighbour (the row owner) holds a slot for
        const uint64_t mj = smask_of(a.smask, a.owner[e]);
        const uint64_t joined = (a.skip_unjoined ? a.sub[a.col[e]] : ~0ull) & mj;
        double score = 0.0;
        for (int32_t t = 0; t < a.T; ++t) {
            const ctp_t tp = const_tp(a.tp) + t;
            if (!tp->scored || !((joined >> t) & 1ull)) continue;
            const int64_t i = slot_idx(mj, t, a.E, e);
            double first = a.first[i], meshd = a.meshd[i], fail = a.fail[i], inval = inv_on ? a.invalid[i] : 0.0;
            uint8_t fl = a.tflags[i];
#if GSIM_REFRESH_GRAFT_EAGER
            // graftTime with the counters (one memory trip per topic; 8 B more per
            // record outside the mesh)
            const int64_t gr = decay ? a.graft[i] : 0;
#endif
            int64_t mt = 0;
            const uint8_t pc = a.mcnt[i];
            if (pc) {   // deliveries since the last pass precede this decay
                meshd = apply_incs(meshd, pc, tp->mesh_message_deliveries_cap);
                a.meshd[i] = meshd;
                a.mcnt[i] = 0;
            }
            if (decay) {
                double x;
                x = first * tp->first_message_deliveries_decay;  if (x < a.dtz) x = 0.0;
                if (x != first) { first = x; a.first[i] = x; }
                x = meshd * tp->mesh_message_deliveries_decay;   if (x < a.dtz) x = 0.0;
                if (x != meshd) { meshd = x; a.meshd[i] = x; }
                x = fail * tp->mesh_failure_penalty_decay;       if (x < a.dtz) x = 0.0;
                if (x != fail) { fail = x; a.fail[i] = x; }
                x = inval * tp->invalid_message_deliveries_decay; if (x < a.dtz) x = 0.0;
                if (x != inval) { inval = x; a.invalid[i] = x; }
                if (fl & GSIM_TF_IN_MESH) {
#if GSIM_REFRESH_GRAFT_EAGER
                    mt = a.now - gr;
#else
                    mt = a.now - a.graft[i];
#endif
                    // lazy meshTime: derived from graftTime and
                    // this refresh's clock where it is read (lazy_mtime)
                    if (!a.mt_lazy || mt < 0) a.mtime[i] = mt;
                    if (mt > tp->mesh_message_deliveries_activation_ns && !(fl & GSIM_TF_ACTIVE)) {
                        fl |= GSIM_TF_ACTIVE;
                        a.tflags[i] = fl;
                    }
                } else if (!a.mt_lazy) {
                    // 0 outside the mesh, unobservable there; in
                    // lazy mode every exit from the mesh stored the 0 itself
                    a.mtime[i] = 0;
                }
            } else if (SCORE && (fl & GSIM_TF_IN_MESH)) {
                const int64_t g = conn && a.mt_lazy ? a.graft[i] : INT64_MAX;
                mt = g <= a.mt_R ? a.mt_R - g : a.mtime[i];
            }
            if (REFRESH && inval != 0.0) inv_left = true;
            if (SCORE) {
                double ts = 0.0;
                if (fl & GSIM_TF_IN_MESH) {                               // P1
                    double p1 = 0.0;
                    if (tp->time_in_mesh_quantum_ns != 0) p1 = (double)go_div(mt, tp->time_in_mesh_quantum_ns);
                    if (p1 > tp->time_in_mesh_cap) p1 = tp->time_in_mesh_cap;
                    ts += p1 * tp->time_in_mesh_weight;
                }
                ts += first * tp->first_message_deliveries_weight;         // P2
                if (fl & GSIM_TF_ACTIVE) {                                 // P3
                    if (meshd < tp->mesh_message_deliveries_threshold) {
                        const double deficit = tp->mesh_message_deliveries_threshold - meshd;
                        const double p3 = deficit * deficit;
                        ts += p3 * tp->mesh_message_deliveries_weight;
                    }
                }
                ts += fail * tp->mesh_failure_penalty_weight;              // P3b
                const double p4 = inval * inval;                           // P4
                ts += p4 * tp->invalid_message_deliveries_weight;
                score += ts * tp->topic_weight;
            }
        }
        double bp = a.bp[e];
        if (decay) {
            double x = bp * a.bp_decay;
            if (x < a.dtz) x = 0.0;
            if (x != bp) { bp = x; a.bp[e] = x; }
        }
        if (REFRESH) {
            // broken IWANT promises of the heartbeat that follows this decay
            // (applyIwantPenalties -> AddPenalty, gossipsub.go:1620-1625)
            const uint8_t pn = a.pen[e];
            if (pn) { bp = bp + (double)pn; a.bp[e] = bp; a.pen[e] = 0; }
        }
        if (SCORE) {
            if (a.topic_cap > 0 && score > a.topic_cap) score = a.topic_cap;
            const double p5 = a.p5[a.owner[e]];                           // P5 (neighbour = row owner)
            score += p5 * a.w5;
            score += a.p6[e] * a.w6;                                       // P6
            if (bp > a.bp_thr) {                                           // P7
                const double excess = bp - a.bp_thr;
                const double p7 = excess * excess;
                score += p7 * a.w7;
            }
            a.score[e] = score;
        }
    }
    if (REFRESH && a0.inv_next && __ballot(inv_left) && (threadIdx.x & 63) == 0) *a0.inv_next = 1u;
}

// ---------------------------------------------------------------------------
// Kernel 2: ipColocationFactor (score.go:344-388) as a segmented count over
// each observer's row keyed by IP id.  Only re-run when the tracked set or the
// IP assignment changes (AddPeer/RemovePeer/purge), not every heartbeat.
// One observer row per lane group (the heartbeat's row classes: W = 16 / 32
// / 64 lanes for rows of at most W connections), lane l = the row's l-th
// connection.  Each lane forms its member's IP key: the neighbour's IP id when
// the neighbour is tracked and has exactly one IP (the common case), else a
// sentinel (untracked / no IP / several IPs).  A member's count for its IP is
// the number of equal keys in the group, W shuffles in registers.  A row with a
// several-IP member counts per IP of the neighbour over the row from memory,
// walking a member's IP list only when it has several.  The counts and the
// order of the sum are the reference's per-IP loop (score.go:344-388); the
// result is the P6 value of record rev[e].  Hub rows (more than 64
// connections): k_ip_colocation_hub.
constexpr uint32_t kIpUntracked = 0xFFFFFFFFu, kIpMulti = 0xFFFFFFFEu, kIpNone = 0xFFFFFFFDu;

__device__ __forceinline__ uint32_t ip_key(const ColocArgs& a, uint32_t e)
{
    if (!(a.estate[a.rev[e]] & GSIM_ES_TRACKED)) return kIpUntracked;
    const uint32_t j = a.col[e];
    const uint32_t q0 = a.ip_ptr[j], q1 = a.ip_ptr[j + 1];
    return q1 == q0 ? kIpNone : q1 - q0 == 1 ? a.ip_ids[q0] : kIpMulti;
}

// several-IP rows: the per-IP count of member e's neighbour over the row [b, en)
__device__ double p6_scan(const ColocArgs& a, uint32_t b, uint32_t en, uint32_t e)
{
    double res = 0.0;
    const uint32_t j = a.col[e];
    for (uint32_t q = a.ip_ptr[j]; q < a.ip_ptr[j + 1]; ++q) {
        const uint32_t ip = a.ip_ids[q];
        if (a.ip_white && a.ip_white[ip]) continue;
        int32_t cnt = 0;
        for (uint32_t e2 = b; e2 < en; ++e2) {
            if (!(a.estate[a.rev[e2]] & GSIM_ES_TRACKED)) continue;
            const uint32_t j2 = a.col[e2];
            for (uint32_t q2 = a.ip_ptr[j2]; q2 < a.ip_ptr[j2 + 1]; ++q2)
                if (a.ip_ids[q2] == ip) { ++cnt; break; }
        }
        if (cnt > a.thr) {
            const double surplus = (double)(cnt - a.thr);
            res += surplus * surplus;
        }
    }
    return res;
}

__device__ __forceinline__ double p6_of(const ColocArgs& a, uint32_t k, int32_t cnt)
{
    if (k >= kIpNone || (a.ip_white && a.ip_white[k]) || cnt <= a.thr) return 0.0;   // no IP, untracked, whitelisted
    const double surplus = (double)(cnt - a.thr);
    return surplus * surplus;
}

template <int W>
__global__ __launch_bounds__(256) void k_ip_coloc_rows(ColocArgs a, const uint32_t* rows, int64_t nrows, int64_t base)
{
    if (a.gate && *a.gate == 0) return;
    constexpr int G = 64 / W;
    const int lane = threadIdx.x & 63, gl = lane % W;
    const int64_t ngroups = (nrows + G - 1) / G * G;
    for (int64_t x = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / W; x < ngroups; x += (int64_t)gridDim.x * blockDim.x / W) {
        bool row_ok = x < nrows;
        const uint32_t i = row_ok ? (rows ? rows[x] : (uint32_t)(base + x)) : 0u;
        if (row_ok && a.rowflag) {                                // only rows whose tracked set changed
            row_ok = a.rowflag[i] != 0;
            if (row_ok && gl == 0) a.rowflag[i] = 0;
        }
        const uint32_t b = row_ok ? a.row_ptr[i] : 0u, deg = row_ok ? a.row_ptr[i + 1] - b : 0u;
        const bool on = (uint32_t)gl < deg;
        const uint32_t e = b + (uint32_t)gl;
        const uint32_t k = on ? ip_key(a, e) : kIpUntracked;
        const uint64_t gm = W == 64 ? ~0ull : (((1ull << W) - 1ull) << (lane - gl));
        const bool multi = (__ballot(k == kIpMulti) & gm) != 0;
        int32_t cnt = 0;
#pragma unroll 16
        for (int q = 0; q < W; ++q) {
            const uint32_t kq = (uint32_t)__shfl((int)k, q, W);
            cnt += (q < (int)deg && kq == k) ? 1 : 0;
        }
        if (!on) continue;
        a.p6[a.rev[e]] = multi ? (k == kIpUntracked ? 0.0 : p6_scan(a, b, b + deg, e)) : p6_of(a, k, cnt);
    }
}

// Hub rows (more than hub_min connections, the heartbeat's hub classes):
// one block per row.  The row's keys are staged in LDS; when every tracked
// member has at most one IP they are sorted (bitonic) and each member's count
// is an equal range of its IP, O(deg log deg) instead of O(deg^2) (a
// 4096-connection row: 1.7e7 key loads); a row with a several-IP member
// counts per IP from memory (p6_scan).  Rows longer than kHubP6Max (the
// reference's ipColocationFactor has no degree bound, score.go:344-388) are
// counted in tiles: per chunk of kHubP6Max members (their keys and counts in
// LDS), every kHubP6Max-key tile of the row is sorted in turn and each member
// adds its key's range in the tile -- the same counts, tiles^2 sorts.
constexpr int kHubP6Max = 4096;

__device__ __forceinline__ void bitonic_sort_lds(uint32_t* s, uint32_t n2)
{
    for (uint32_t k = 2; k <= n2; k <<= 1)               // bitonic sort, ascending
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t q = threadIdx.x; q < n2; q += blockDim.x) {
                const uint32_t p = q ^ j;
                if (p > q) {
                    const uint32_t u = s[q], v = s[p];
                    if (((q & k) == 0) ? (u > v) : (u < v)) { s[q] = v; s[p] = u; }
                }
            }
            __syncthreads();
        }
}

// occurrences of key k in the sorted s[0, n2)
__device__ __forceinline__ int32_t sorted_count(const uint32_t* s, uint32_t n2, uint32_t k)
{
    uint32_t lo = 0, hi = n2;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (s[m] < k) lo = m + 1; else hi = m; }
    uint32_t lo2 = lo, hi2 = n2;
    while (lo2 < hi2) { const uint32_t m = (lo2 + hi2) >> 1; if (s[m] <= k) lo2 = m + 1; else hi2 = m; }
    return (int32_t)(lo2 - lo);
}

__global__ __launch_bounds__(256) void k_ip_colocation_hub(ColocArgs a, const uint32_t* rows, int64_t nrows)
{
    if (a.gate && *a.gate == 0) return;
    __shared__ uint32_t s_key[kHubP6Max];    // the members' keys (a chunk of them on a longer row)
    __shared__ uint32_t s_srt[kHubP6Max];    // a sorted key tile
    __shared__ int32_t s_cnt[kHubP6Max];     // the members' counts over the tiles so far
    for (int64_t x = blockIdx.x; x < nrows; x += gridDim.x) {
        const uint32_t i = rows[x];
        const uint32_t b = a.row_ptr[i], deg = a.row_ptr[i + 1] - b;
        if (deg <= a.hub_min) continue;
        if (a.sharded && (i < a.olo || i >= a.ohi)) continue;
        if (a.rowflag && !a.rowflag[i]) continue;               // only rows whose tracked set changed
        __syncthreads();                                          // (every thread has read the flag)
        if (a.rowflag && threadIdx.x == 0) a.rowflag[i] = 0;
        const bool one_tile = deg <= (uint32_t)kHubP6Max;
        bool multi = false;
        for (uint32_t q = threadIdx.x; q < deg; q += blockDim.x) {
            const uint32_t k = ip_key(a, b + q);
            if (one_tile) s_key[q] = k;
            multi |= k == kIpMulti;
        }
        if (!__syncthreads_or(multi)) {
            for (uint32_t mc = 0; mc < deg; mc += kHubP6Max) {    // member chunks
                const uint32_t nm = deg - mc < (uint32_t)kHubP6Max ? deg - mc : (uint32_t)kHubP6Max;
                for (uint32_t q = threadIdx.x; q < nm; q += blockDim.x) {
                    if (!one_tile) s_key[q] = ip_key(a, b + mc + q);
                    s_cnt[q] = 0;
                }
                for (uint32_t tc = 0; tc < deg; tc += kHubP6Max) {  // key tiles
                    const uint32_t nk = deg - tc < (uint32_t)kHubP6Max ? deg - tc : (uint32_t)kHubP6Max;
                    uint32_t n2 = 1;
                    while (n2 < nk) n2 <<= 1;
                    __syncthreads();                              // (s_srt of the last tile is read)
                    for (uint32_t q = threadIdx.x; q < n2; q += blockDim.x)
                        s_srt[q] = q >= nk ? 0xFFFFFFFFu : one_tile ? s_key[q] : ip_key(a, b + tc + q);
                    __syncthreads();
                    bitonic_sort_lds(s_srt, n2);
                    for (uint32_t q = threadIdx.x; q < nm; q += blockDim.x) {
                        const uint32_t k = s_key[q];
                        if (k < kIpNone) s_cnt[q] += sorted_count(s_srt, n2, k);
                    }
                }
                for (uint32_t q = threadIdx.x; q < nm; q += blockDim.x)
                    a.p6[a.rev[b + mc + q]] = p6_of(a, s_key[q], s_cnt[q]);
                __syncthreads();                                  // s_key is rewritten by the next chunk
            }
        } else {
            for (uint32_t q = threadIdx.x; q < deg; q += blockDim.x) {
                const uint32_t k = one_tile ? s_key[q] : ip_key(a, b + q);
                a.p6[a.rev[b + q]] = k == kIpUntracked ? 0.0 : p6_scan(a, b, b + deg, b + q);
            }
        }
        __syncthreads();                                          // LDS is rewritten by the next row
    }
}

// SetTopicScoreParams recap (score.go:224-238) of topic t.
__global__ __launch_bounds__(256) void k_recap(int64_t E, const uint8_t* estate, const uint32_t* owner,
                                               const uint64_t* smask, int32_t t, double* first, double* meshd,
                                               double first_cap, double mesh_cap, int do_first, int do_mesh)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) {
        if (!(estate[e] & GSIM_ES_TRACKED)) continue;
        const uint64_t m = smask_of(smask, owner[e]);
        if (!slot_has(m, t)) continue;
        const int64_t i = slot_idx(m, t, E, e);
        if (do_first && first[i] > first_cap) first[i] = first_cap;
        if (do_mesh && meshd[i] > mesh_cap) meshd[i] = mesh_cap;
    }
}

// Apply every pending meshd increment (before the counter is read through the
// ABI or its cap changes).
__global__ __launch_bounds__(256) void k_apply_mcnt(ScoreArgs a)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t total = a.E * (int64_t)a.S;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const uint8_t n = a.mcnt[x];
        if (!n) continue;
        const int32_t p = (int32_t)(x / a.E);
        const int32_t t = a.smask ? slot_topic(a.smask[a.owner[x - (int64_t)p * a.E]], p) : p;
        if (t < 0) continue;
        a.meshd[x] = apply_incs(a.meshd[x], n, const_tp(a.tp)[t].mesh_message_deliveries_cap);
        a.mcnt[x] = 0;
    }
}

// Store every lazy meshTime (lazy_mtime): the records the refresh pass
// rewrites (tracked, connected, owned, scored topics) get R - graftTime in the
// mesh and 0 outside it, the others keep what they hold.
__global__ __launch_bounds__(256) void k_mtime_materialize(ScoreArgs a)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.E; e += stride) {
        if (a.sharded) {
            const uint32_t o = a.col[e];
            if (o < a.olo || o >= a.ohi) continue;
        }
        const uint8_t st = a.estate[e];
        if ((st & (GSIM_ES_TRACKED | GSIM_ES_CONNECTED)) != (GSIM_ES_TRACKED | GSIM_ES_CONNECTED)) continue;
        const uint64_t mj = smask_of(a.smask, a.owner[e]);
        for (int32_t t = 0; t < a.T; ++t) {
            if (!const_tp(a.tp)[t].scored || !slot_has(mj, t)) continue;
            const int64_t i = slot_idx(mj, t, a.E, e);
            const int64_t old = a.mtime[i];
            const int64_t v = (a.tflags[i] & GSIM_TF_IN_MESH) ? lazy_mtime(1, a.mt_R, a.graft[i], old) : 0;
            if (v != old) a.mtime[i] = v;
        }
    }
}

// Seeded synthetic steady-state-like counters for benchmarking at full size
// (SURVEY.md §8(d)): a Philox draw per edge-topic record decides mesh
// membership (probability D/k), activation, graft time and the four counters.
__global__ __launch_bounds__(256) void k_fill_synthetic(ScoreArgs a, uint64_t seed, double p_mesh)
{
    // thread per observer edge e of the owned rows; its record lives at r =
    // rev[e].  The draws are keyed by the global edge index, so a sharded
    // network gets the same state as the whole one.
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const double inv = 1.0 / 4294967296.0;
    for (int64_t e = a.e_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.e_hi; e += stride) {
        const int64_t r = a.rev[e];
        const int64_t ge = a.geid_base + (e - a.e_lo);
        // topics both endpoints joined: only there can a mesh link or
        // deliveries exist (owner[e] = observer, owner[r] = neighbour)
        const uint64_t shared = a.sub ? a.sub[a.owner[e]] & a.sub[a.owner[r]] : ~0ull;
        // topic slots: the router state of edge e is the observer's (owner[e]),
        // the record r the neighbour's row's (owner[r])
        const uint64_t mi = smask_of(a.smask, a.owner[e]), mj = smask_of(a.smask, a.owner[r]);
        for (int32_t t = 0; t < a.T; ++t) {
            const int64_t i = slot_idx(mi, t, a.E, e);
            const int64_t ir = slot_idx(mj, t, a.E, r);
            if (!((shared >> t) & 1ull)) {
                if (slot_has(mj, t)) {
                    a.tflags[ir] = 0; a.graft[ir] = 0; a.mtime[ir] = 0;
                    a.first[ir] = 0.0; a.meshd[ir] = 0.0; a.fail[ir] = 0.0; a.invalid[ir] = 0.0;
                }
                if (slot_has(mi, t)) a.mflags[i] = 0;
                continue;
            }
            const int64_t gi = (int64_t)t * a.E_glob + ge;
            const u32x4 x = philox4x32_10((uint32_t)gi, (uint32_t)(gi >> 32), 0x5eed, 1, k0, k1);
            const u32x4 q = philox4x32_10((uint32_t)gi, (uint32_t)(gi >> 32), 0x5eed, 2, k0, k1);
            const bool in_mesh = x.x * inv < p_mesh;
            uint8_t fl = in_mesh ? GSIM_TF_IN_MESH : 0;
            if (in_mesh && (x.y & 15) != 0) fl |= GSIM_TF_ACTIVE;
            a.tflags[ir] = fl;
            a.mflags[i] = in_mesh ? GSIM_TF_MESH : 0;
            const int64_t g = in_mesh ? a.now - (int64_t)(x.z % 3600u) * 1000000000LL : 0;
            a.graft[ir] = g;
            a.mtime[ir] = in_mesh ? a.now - g : 0;
            a.first[ir] = (double)(q.x % 2000u) * 0.25;
            a.meshd[ir] = in_mesh ? (double)(q.y % 1600u) * 0.25 : 0.0;
            a.fail[ir] = (q.z & 7) == 0 ? (double)(q.z % 4000u) * 0.125 : 0.0;
            a.invalid[ir] = (q.w & 511) == 0 ? (double)(q.w % 64u) * 0.125 : 0.0;
        }
        const u32x4 b = philox4x32_10((uint32_t)ge, (uint32_t)(ge >> 32), 0x5eed, 3, k0, k1);
        a.bp[r] = (b.x & 15) == 0 ? (double)(b.y % 100u) * 0.125 : 0.0;
        a.estate[r] = GSIM_ES_TRACKED | GSIM_ES_CONNECTED;
        a.expire[r] = 0;
        a.rstate[e] = GSIM_ES_CONNECTED;
    }
}

// Aggregate state census (counts per category, see gsim_census in gsim.h).
__global__ __launch_bounds__(256) void k_census(ScoreArgs a, unsigned long long* out)
{
    unsigned long long c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.E; e += stride) {
        if (a.sharded && (a.col[e] < a.olo || a.col[e] >= a.ohi)) continue;   // another shard's record
        const uint8_t st = a.estate[e];
        if (!(st & GSIM_ES_TRACKED)) continue;
        c[7] += 1;
        if (!(st & GSIM_ES_CONNECTED)) continue;
        const uint64_t mj = smask_of(a.smask, a.owner[e]);
        const uint64_t joined = (a.skip_unjoined ? a.sub[a.col[e]] : ~0ull) & mj;   // records the score pass reads
        for (int32_t t = 0; t < a.T; ++t) {
            if (!const_tp(a.tp)[t].scored || !((joined >> t) & 1ull)) continue;
            const int64_t i = slot_idx(mj, t, a.E, e);
            const uint8_t fl = a.tflags[i];
            c[0] += 1;
            c[1] += (fl & GSIM_TF_IN_MESH) != 0;
            c[2] += a.first[i] != 0.0;
            c[3] += apply_incs(a.meshd[i], a.mcnt[i], const_tp(a.tp)[t].mesh_message_deliveries_cap) != 0.0;
            c[4] += a.fail[i] != 0.0;
            c[5] += a.invalid[i] != 0.0;
        }
    }
    for (int64_t e = a.e_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.e_hi; e += stride) {
        if (!(a.rstate[e] & GSIM_ES_CONNECTED)) continue;   // router mesh links (edge order), owned rows
        const uint64_t mi = smask_of(a.smask, a.owner[e]);
        for (int32_t t = 0; t < a.T; ++t)
            if (slot_has(mi, t)) c[6] += (a.mflags[slot_idx(mi, t, a.E, e)] & GSIM_TF_MESH) != 0;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        unsigned long long v = c[k];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&out[k], v);
    }
}

// Layout permutations between the ABI's edge-order view and record order
// (DESIGN.md §2).  rev is an involution, so one gather serves both ways.
template <typename T>
__global__ __launch_bounds__(256) void k_gather_rev(const T* __restrict__ in, T* __restrict__ out,
                                                    const uint32_t* __restrict__ rev, int64_t E, int64_t total)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const int64_t p = x / E, e = x - p * E;
        out[x] = in[p * E + rev[e]];
    }
}

// The ABI's dense view [npar][T][E] (edge order) of a topic-slot array
// [npar][S][E]: view index e of topic t is device index
// x = rev[e] (record order; rev == nullptr: edge order), in the plane of t's
// slot of x's row owner.  Entries outside the masks read as zero.
template <typename T>
__global__ __launch_bounds__(256) void k_view_read(const T* __restrict__ dev, T* __restrict__ view,
                                                   const uint32_t* rev, const uint32_t* owner, const uint64_t* smask,
                                                   int64_t E, int32_t nT, int32_t S, int64_t total)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t TE = (int64_t)nT * E;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += stride) {
        const int64_t par = v / TE, rem = v - par * TE;
        const int32_t t = (int32_t)(rem / E);
        const int64_t e = rem - (int64_t)t * E;
        const int64_t x = rev ? (int64_t)rev[e] : e;
        const uint64_t m = smask_of(smask, owner[x]);
        view[v] = slot_has(m, t) ? dev[par * (int64_t)S * E + slot_idx(m, t, E, x)] : (T)0;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_view_write(const T* __restrict__ view, T* __restrict__ dev,
                                                    const uint32_t* rev, const uint32_t* owner, const uint64_t* smask,
                                                    int64_t E, int32_t nT, int32_t S, int64_t total)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t TE = (int64_t)nT * E;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += stride) {
        const int64_t par = v / TE, rem = v - par * TE;
        const int32_t t = (int32_t)(rem / E);
        const int64_t e = rem - (int64_t)t * E;
        const int64_t x = rev ? (int64_t)rev[e] : e;
        const uint64_t m = smask_of(smask, owner[x]);
        if (slot_has(m, t)) dev[par * (int64_t)S * E + slot_idx(m, t, E, x)] = view[v];
    }
}

// The slots a written view needs: bit t for both endpoints of every edge
// with a non-zero entry (a mesh link, control or record of a topic implies
// both ends hold it; a record lives in one endpoint's row, the router state
// in the other's, and replies go back the other way).
template <typename T>
__global__ __launch_bounds__(256) void k_view_need(const T* __restrict__ view, const uint32_t* rev,
                                                   const uint32_t* owner, int64_t E, int32_t nT, int64_t total,
                                                   unsigned long long* need)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t TE = (int64_t)nT * E;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += stride) {
        const T val = view[v];
        if (val == (T)0) continue;
        const int64_t par = v / TE, rem = v - par * TE;
        const int32_t t = (int32_t)(rem / E);
        const int64_t e = rem - (int64_t)t * E;
        const unsigned long long bit = 1ull << t;
        atomicOr(&need[owner[e]], bit);
        atomicOr(&need[owner[rev[e]]], bit);
    }
}

__global__ __launch_bounds__(256) void k_tflags_compose(const uint8_t* rec, const uint8_t* mf, uint8_t* out,
                                                        const uint32_t* rev, const uint32_t* owner,
                                                        const uint64_t* smask, int64_t E, int64_t total)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
        const int32_t t = (int32_t)(x / E);
        const int64_t e = x - (int64_t)t * E, r = rev[e];
        const uint64_t mr = smask_of(smask, owner[r]), me = smask_of(smask, owner[e]);
        const uint8_t a = slot_has(mr, t) ? rec[slot_idx(mr, t, E, r)] : 0;
        const uint8_t b = slot_has(me, t) ? mf[slot_idx(me, t, E, e)] : 0;
        out[x] = (uint8_t)((a & (GSIM_TF_IN_MESH | GSIM_TF_ACTIVE)) | (b & (GSIM_TF_MESH | GSIM_TF_FANOUT)));
    }
}

__global__ __launch_bounds__(256) void k_tflags_split(const uint8_t* in, uint8_t* rec, uint8_t* mf,
                                                      const uint32_t* rev, const uint32_t* owner,
                                                      const uint64_t* smask, int64_t E, int64_t total)
{
    // thread per (t, x): x both the record index (score bits of view entry
    // rev[x]) and the edge index (router bits of view entry x)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += stride) {
        const int32_t t = (int32_t)(v / E);
        const int64_t x = v - (int64_t)t * E;
        const uint64_t m = smask_of(smask, owner[x]);
        if (!slot_has(m, t)) continue;
        const int64_t i = slot_idx(m, t, E, x);
        rec[i] = (uint8_t)(in[(int64_t)t * E + rev[x]] & (GSIM_TF_IN_MESH | GSIM_TF_ACTIVE));
        mf[i] = (uint8_t)(in[v] & (GSIM_TF_MESH | GSIM_TF_FANOUT));
    }
}

// Re-layout of a topic-slot array [npar][S0][E] -> [npar][S1][E] when slot
// masks grow (ensure_slots): old mask m0, new m1 of each row owner.
template <typename T>
__global__ __launch_bounds__(256) void k_slot_relayout(const T* __restrict__ src, T* __restrict__ dst,
                                                       const uint32_t* owner, const uint64_t* m0s, const uint64_t* m1s,
                                                       int64_t E, int32_t S0, int32_t S1, int32_t npar)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < E; x += stride) {
        const uint32_t o = owner[x];
        const uint64_t m0 = smask_of(m0s, o), m1 = smask_of(m1s, o);
        for (int32_t par = 0; par < npar; ++par) {
            const T* s0 = src + (int64_t)par * S0 * E;
            T* s1 = dst + (int64_t)par * S1 * E;
            int32_t p1 = 0;
            for (uint64_t b = m1; b; b &= b - 1, ++p1) {
                const int32_t t = __builtin_ctzll(b);
                s1[(int64_t)p1 * E + x] = slot_has(m0, t) ? s0[slot_idx(m0, t, E, x)] : (T)0;
            }
            for (; p1 < S1; ++p1) s1[(int64_t)p1 * E + x] = (T)0;
        }
    }
}

__global__ __launch_bounds__(256) void k_estate_split(const uint8_t* in, uint8_t* rec, uint8_t* rs,
                                                      const uint32_t* rev, int64_t E)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) {
        rec[e] = in[rev[e]];
        rs[e] = (uint8_t)(in[e] & GSIM_ES_CONNECTED);
    }
}

// Delivery state of every edge index e (GSIM_DS_*): the router's connected
// bit of edge e, and of record e the AcceptFrom verdict (gossipsub.go:598-609:
// score snapshot >= graylistThreshold) and whether it is tracked.
__global__ __launch_bounds__(256) void k_delivery_state(const double* score, const uint8_t* estate,
                                                        const uint8_t* rstate, const uint8_t* direct,
                                                        const uint32_t* rev, uint8_t* ds, int64_t E, double gray)
{
    // AcceptFrom is the receiver's: its direct peers are accepted whatever
    // their score (gossipsub.go:598-609); its flag for the sender sits at rev[r]
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < E; r += stride)
        ds[r] = (uint8_t)(((rstate[r] & GSIM_ES_CONNECTED) ? GSIM_DS_CONNECTED : 0) |
                          ((score[r] >= gray || direct[rev[r]]) ? GSIM_DS_ACCEPT : 0) |
                          ((estate[r] & GSIM_ES_TRACKED) ? GSIM_DS_TRACKED : 0) |
                          (direct[r] ? GSIM_DS_DIRECT : 0));
}

__global__ void k_fill_u8(uint8_t* p, int64_t n, uint8_t v)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

// ---------------------------------------------------------------------------
// host side

namespace {

int grid_for(int64_t n, int block = 256, int cap = 16384)
{
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

template <typename T>
int dalloc(gsim_handle* h, T** p, int64_t n)
{
    *p = nullptr;
    if (n <= 0) n = 1;
    hipError_t e = hipMalloc((void**)p, sizeof(T) * (size_t)n);
    if (e != hipSuccess) {
        h->err = std::string("hipMalloc failed: ") + hipGetErrorString(e);
        return GSIM_ENOMEM;
    }
    h->bytes_allocated += sizeof(T) * (size_t)n;
    return GSIM_OK;
}

template <typename T>
void dfree(T*& p)
{
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

}  // namespace

int hip_check(gsim_handle* h, hipError_t e, const char* what)
{
    if (e == hipSuccess) return GSIM_OK;
    h->err = std::string(what) + ": " + hipGetErrorString(e);
    return GSIM_EDEVICE;
}

void free_graph(gsim_handle* h)
{
    dfree(h->d_row_ptr); dfree(h->d_col); dfree(h->d_rev); dfree(h->d_owner);
    dfree(h->d_sub); dfree(h->d_outbound); dfree(h->d_direct);
    dfree(h->d_ip_ptr); dfree(h->d_ip_ids); dfree(h->d_ip_white); dfree(h->d_p5);
    dfree(h->d_first); dfree(h->d_meshd); dfree(h->d_fail); dfree(h->d_invalid);
    dfree(h->d_graft); dfree(h->d_mtime); dfree(h->d_tflags); dfree(h->d_mflags);
    dfree(h->d_bp); dfree(h->d_estate); dfree(h->d_expire); dfree(h->d_p6); dfree(h->d_p6row); dfree(h->d_churn); h->churn_cap = 0; dfree(h->d_churn_mark); dfree(h->d_score);
    dfree(h->d_backoff); dfree(h->d_rstate); dfree(h->d_dstate); dfree(h->d_mcnt); dfree(h->d_pen);
    dfree(h->d_smask);
    h->smask.clear();
    h->S = 0;
    h->bytes_allocated = 0;
    h->n = h->e = 0;
}

// any counter may be non-zero (state written through the ABI, a fill, new
// parameters): the next refresh reads the invalid planes and settles the flag
static hipError_t inv_mark_all(gsim_handle* h)
{
    return hipMemsetAsync(h->d_inv_live, 1, 2 * sizeof(uint32_t), h->stream);
}

static ScoreArgs make_score_args(gsim_handle* h, int64_t now)
{
    ScoreArgs a{};
    a.E = h->e;
    a.T = h->t;
    a.sub = h->d_sub;
    a.col = h->d_col;
    a.smask = h->d_smask;
    a.S = h->S;
    // (the subscription gather costs ≈1 ms per pass at C3, where nothing is skipped)
    a.skip_unjoined = (h->unjoined_zero && !h->all_joined) ? 1 : 0;
    a.tp = h->d_tp;
    a.dtz = h->pp.decay_to_zero;
    a.bp_decay = h->pp.behaviour_penalty_decay;
    a.topic_cap = h->pp.topic_score_cap;
    a.w5 = h->pp.app_specific_weight;
    a.w6 = h->pp.ip_colocation_factor_weight;
    a.bp_thr = h->pp.behaviour_penalty_threshold;
    a.w7 = h->pp.behaviour_penalty_weight;
    a.owner = h->d_owner;
    a.p5 = h->d_p5;
    a.first = h->d_first; a.meshd = h->d_meshd; a.fail = h->d_fail; a.invalid = h->d_invalid;
    a.mcnt = h->d_mcnt;
    a.graft = h->d_graft; a.mtime = h->d_mtime; a.tflags = h->d_tflags;
    a.mflags = h->d_mflags; a.rstate = h->d_rstate; a.rev = h->d_rev;
    a.bp = h->d_bp; a.pen = h->d_pen; a.estate = h->d_estate; a.expire = h->d_expire; a.p6 = h->d_p6; a.score = h->d_score;
    a.now = now;
    a.mt_lazy = h->mt_lazy ? 1 : 0;
    a.mt_R = h->mt_R;
    a.purged = h->d_flags;
    a.p6row = h->d_p6row;
    a.sharded = h->sh ? 1 : 0;
    a.olo = (uint32_t)h->olo();
    a.ohi = (uint32_t)h->ohi();
    a.e_lo = h->sh ? h->sh->own_e_lo : 0;
    a.e_hi = h->sh ? h->sh->own_e_hi : h->e;
    a.geid_base = h->sh ? h->sh->geid_base : 0;
    a.E_glob = h->sh ? h->sh->E_global : h->e;
    a.inv_live = h->d_inv_live + (h->inv_par & 1);
    a.inv_next = h->d_inv_live + ((h->inv_par + 1) & 1);
    return a;
}

// Whether an IP id is listed by two different peers (ip_ptr CSR over n peers).
static bool ips_shared(int64_t n, const uint32_t* ip_ptr, const uint32_t* ip_ids, uint32_t n_ips)
{
    if (!ip_ptr || !ip_ids || n_ips == 0) return false;
    std::vector<int64_t> owner((size_t)n_ips, -1);
    for (int64_t i = 0; i < n; ++i)
        for (uint32_t q = ip_ptr[i]; q < ip_ptr[i + 1]; ++q) {
            int64_t& o = owner[ip_ids[q]];
            if (o >= 0 && o != i) return true;
            o = i;
        }
    return false;
}

int launch_ip_colocation(gsim_handle* h, const int32_t* gate)
{
    ProfScope ps(h, GSIM_K_IP_COLOCATION);
    if (!h->ip_shared && h->pp.ip_colocation_factor_threshold >= 1) {
        // every IP is one peer's: peersInIP - threshold <= 0 for every record
        // (score.go:426-446), P6 = 0 -- as the scan computes, without it (c5
        // with one IP per peer: 11 ms per tick)
        hipError_t e = hipMemsetAsync(h->d_p6, 0, sizeof(double) * (size_t)h->e, h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(h->d_p6row, 0, (size_t)h->n, h->stream);
        h->p6_dirty = false;
        h->p6_rows_only = false;
        return hip_check(h, e, "P6 (no shared IP)");
    }
    ColocArgs c{};
    c.gate = gate;
    c.E = h->e; c.row_ptr = h->d_row_ptr; c.col = h->d_col; c.rev = h->d_rev; c.owner = h->d_owner;
    c.ip_ptr = h->d_ip_ptr; c.ip_ids = h->d_ip_ids; c.ip_white = h->has_white ? h->d_ip_white : nullptr;
    c.estate = h->d_estate; c.p6 = h->d_p6; c.thr = h->pp.ip_colocation_factor_threshold;
    c.sharded = h->sh ? 1 : 0;
    c.olo = (uint32_t)h->olo();
    c.ohi = (uint32_t)h->ohi();
    c.hub_min = 64u;
    // churn / purges changed some rows' tracked sets: those rows alone
    c.rowflag = h->p6_rows_only ? h->d_p6row : nullptr;
    // the heartbeat's row classes: owned observers by row length
    RowClasses rc{};
    row_classes(h, &rc);
    auto grid = [](int64_t groups, int per_block) {
        return dim3((uint32_t)std::max<int64_t>(1, std::min<int64_t>((groups + per_block - 1) / per_block, 65536)));
    };
    if (!rc.rows) {                          // one class: the owned rows [olo, ohi) in order
        const int64_t n = h->ohi() - h->olo();
        if (rc.n16 == n) hipLaunchKernelGGL(k_ip_coloc_rows<16>, grid(n, 16), dim3(256), 0, h->stream, c, nullptr, n, h->olo());
        else if (rc.n32 == n) hipLaunchKernelGGL(k_ip_coloc_rows<32>, grid(n, 8), dim3(256), 0, h->stream, c, nullptr, n, h->olo());
        else hipLaunchKernelGGL(k_ip_coloc_rows<64>, grid(n, 4), dim3(256), 0, h->stream, c, nullptr, n, h->olo());
    } else {
        if (rc.n16) hipLaunchKernelGGL(k_ip_coloc_rows<16>, grid(rc.n16, 16), dim3(256), 0, h->stream, c, rc.rows, rc.n16,
                                       (int64_t)0);
        if (rc.n32) hipLaunchKernelGGL(k_ip_coloc_rows<32>, grid(rc.n32, 8), dim3(256), 0, h->stream, c, rc.rows + rc.n16,
                                       rc.n32, (int64_t)0);
        if (rc.n64) hipLaunchKernelGGL(k_ip_coloc_rows<64>, grid(rc.n64, 4), dim3(256), 0, h->stream, c,
                                       rc.rows + rc.n16 + rc.n32, rc.n64, (int64_t)0);
        const int64_t nhub = rc.nhub;
        if (nhub)
            hipLaunchKernelGGL(k_ip_colocation_hub, dim3((uint32_t)std::min<int64_t>(nhub, 65536)), dim3(256), 0,
                               h->stream, c, rc.rows + rc.n16 + rc.n32 + rc.n64, nhub);
    }
    hipError_t e = hipGetLastError();
    // a full pass re-derived every row: no row stays flagged
    if (e == hipSuccess && !c.rowflag) e = hipMemsetAsync(h->d_p6row, 0, (size_t)h->n, h->stream);
    h->p6_dirty = false;
    h->p6_rows_only = true;      // until a change of more than the tracked sets
    return hip_check(h, e, "k_ip_colocation");
}

template <bool REFRESH, bool SCORE>
static void launch_score_kernel(gsim_handle* h, const ScoreArgs& a)
{
    ProfScope ps(h, REFRESH ? GSIM_K_REFRESH_SCORE : GSIM_K_SCORE);
// blocks of the fused refresh (grid-stride over the records): up to 131072, one
// record per thread at C3 (125000 blocks): 6.99 / 7.04 ms against 7.16 / 7.15 at
// 65536 and 7.25 / 7.24 at 32768 (gpurun_out/r05p_c3); round 4: 65536 8.04 ms
// against 8.26 at 16384 and 8.48 at 4096 (gpurun_out/r04pab)
#ifndef GSIM_REFRESH_GRID
#define GSIM_REFRESH_GRID 131072
#endif
    hipLaunchKernelGGL((k_refresh_score<REFRESH, SCORE>), dim3(grid_for(h->e, 256, GSIM_REFRESH_GRID)), dim3(256), 0,
                       h->stream, a);
}

int launch_refresh_scores(gsim_handle* h, int64_t now)
{
    int rc0 = deliver_flush(h);   // the last round's first deliveries precede the decay
    if (!rc0) rc0 = gater_decay(h, now);              // the peer gater's decayStats
    if (!rc0) rc0 = deliver_promise_check(h, now);   // broken promises of this heartbeat
    if (rc0) return rc0;
    ScoreArgs a = make_score_args(h, now);
    if (h->p6_dirty) {
        int rc = launch_ip_colocation(h);
        if (rc) return rc;
    }
    if (h->maybe_retained) {
        // a purge inside refresh changes the tracked set, so P6 must be
        // re-derived between decay and scoring (score.go:514 removeIPs).
        // The fused pass runs as usual and flags a purge on the device; only
        // then are P6 and every score recomputed (kernels gated on the flag,
        // no host round trip): the same results as refresh, P6 and score in
        // three unconditional passes.
        hipError_t e = hipMemsetAsync(h->d_flags + 1, 0, sizeof(int32_t), h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(a.inv_next, 0, sizeof(uint32_t), h->stream);
        if (e != hipSuccess) return hip_check(h, e, "purge flag");
        a.purged = h->d_flags + 1;
        launch_score_kernel<true, true>(h, a);
        h->inv_par ^= 1;
        int rc = launch_ip_colocation(h, h->d_flags + 1);
        if (rc) return rc;
        ScoreArgs b = a;
        b.inv_live = a.inv_next;     // the flag of the decayed state
        b.gate = h->d_flags + 1;
        b.mt_lazy = 1;       // meshTime as the pass above left it
        b.mt_R = now;
        launch_score_kernel<false, true>(h, b);
    } else {
        hipError_t e = hipMemsetAsync(a.inv_next, 0, sizeof(uint32_t), h->stream);
        if (e != hipSuccess) return hip_check(h, e, "invalid-plane flag");
        launch_score_kernel<true, true>(h, a);
        h->inv_par ^= 1;
    }
    h->mt_lazy = true;
    h->mt_R = now;
    h->mcnt_dirty = false;   // the score pass settled every pending count
    deliver_mcnt_applied(h);
    h->score_version++;
    return hip_check(h, hipGetLastError(), "k_refresh_score");
}

int launch_compute_scores(gsim_handle* h)
{
    int rc0 = deliver_flush(h);
    if (rc0) return rc0;
    if (h->p6_dirty) {
        int rc = launch_ip_colocation(h);
        if (rc) return rc;
    }
    ScoreArgs a = make_score_args(h, 0);
    launch_score_kernel<false, true>(h, a);
    h->mcnt_dirty = false;
    h->score_version++;
    return hip_check(h, hipGetLastError(), "k_refresh_score<score>");
}

int refresh_accept(gsim_handle* h)
{
    if (h->acc_version == h->score_version) return GSIM_OK;
    hipLaunchKernelGGL(k_delivery_state, dim3(grid_for(h->e)), dim3(256), 0, h->stream, (const double*)h->d_score,
                       (const uint8_t*)h->d_estate, (const uint8_t*)h->d_rstate, (const uint8_t*)h->d_direct,
                       (const uint32_t*)h->d_rev, h->d_dstate, h->e,
                       h->th.graylist_threshold);
    h->acc_version = h->score_version;
    return hip_check(h, hipGetLastError(), "k_delivery_state");
}

int materialize_mcnt(gsim_handle* h)
{
    if (!h->mcnt_dirty) return GSIM_OK;
    ScoreArgs a = make_score_args(h, 0);
    hipLaunchKernelGGL(k_apply_mcnt, dim3(grid_for(h->e * (int64_t)std::max(1, h->S))), dim3(256), 0, h->stream, a);
    h->mcnt_dirty = false;
    deliver_mcnt_applied(h);
    return hip_check(h, hipGetLastError(), "k_apply_mcnt");
}

int materialize_mtime(gsim_handle* h, bool leave)
{
    if (!h->mt_lazy) return GSIM_OK;
    ScoreArgs a = make_score_args(h, 0);
    hipLaunchKernelGGL(k_mtime_materialize, dim3(grid_for(h->e)), dim3(256), 0, h->stream, a);
    // (a read may stay lazy: the stored values are the derived ones)
    if (leave) h->mt_lazy = false;
    return hip_check(h, hipGetLastError(), "k_mtime_materialize");
}

// Grow the topic slot masks to cover need[]: every topic
// array is re-laid out into S' planes (one array at a time, so the extra
// memory is one array).  Called for the topics an ABI write, a publication
// by a peer outside its topic (fanout) or a Join brings; a dense handle has
// every slot already.
template <typename T>
static int relayout_one(gsim_handle* h, T** p, int32_t npar, const uint64_t* m0, const uint64_t* m1, int32_t S0,
                        int32_t S1)
{
    if (!*p) return GSIM_OK;
    T* q = nullptr;
    hipError_t e = hipMalloc((void**)&q, sizeof(T) * (size_t)npar * (size_t)S1 * (size_t)std::max<int64_t>(h->e, 1));
    if (e != hipSuccess) return hip_check(h, e, "slot re-layout");
    hipLaunchKernelGGL(k_slot_relayout<T>, dim3(grid_for(h->e)), dim3(256), 0, h->stream, (const T*)*p, q,
                       (const uint32_t*)h->d_owner, m0, m1, h->e, S0, S1, npar);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) { (void)hipFree(q); return hip_check(h, e, "k_slot_relayout"); }
    (void)hipFree(*p);
    *p = q;
    h->bytes_allocated += sizeof(T) * (size_t)npar * (size_t)(S1 - S0) * (size_t)h->e;
    return GSIM_OK;
}

int ensure_slots(gsim_handle* h, const uint64_t* need)
{
    if (!h->d_smask || h->smask.empty()) return GSIM_OK;     // dense: every topic has its plane
    const uint64_t tmask = h->t >= 64 ? ~0ull : ((1ull << h->t) - 1);
    std::vector<uint64_t> m1(h->smask);
    bool grown = false;
    int32_t S1 = h->S;
    for (size_t i = 0; i < m1.size(); ++i) {
        const uint64_t x = m1[i] | (need[i] & tmask);
        if (x != m1[i]) { m1[i] = x; grown = true; }
        S1 = std::max(S1, __builtin_popcountll(x));
    }
    if (!grown) return GSIM_OK;
    int rc = deliver_flush(h);
    if (!rc) rc = materialize_mcnt(h);
    if (rc) return rc;
    uint64_t* d1 = nullptr;
    hipError_t e = hipMalloc((void**)&d1, sizeof(uint64_t) * m1.size());
    if (e == hipSuccess) e = hipMemcpyAsync(d1, m1.data(), sizeof(uint64_t) * m1.size(), hipMemcpyHostToDevice, h->stream);
    if (e != hipSuccess) { if (d1) (void)hipFree(d1); return hip_check(h, e, "slot masks"); }
    const uint64_t* d0 = h->d_smask;
    const int32_t S0 = h->S;
    rc = relayout_one(h, &h->d_first, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_meshd, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_fail, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_invalid, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_graft, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_mtime, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_tflags, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_mcnt, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_mflags, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, &h->d_backoff, 1, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, extra_ctl_slot(h), 2, d0, d1, S0, S1);
    if (!rc) rc = relayout_one(h, deliver_gsel_slot(h), 1, d0, d1, S0, S1);
    if (rc) { (void)hipFree(d1); return rc; }
    (void)hipFree(h->d_smask);
    h->d_smask = d1;
    h->smask.swap(m1);
    h->S = S1;
    h->mesh_version++;
    return slots_changed(h);
}

// ---------------------------------------------------------------------------
// C ABI

// Copy a field to the host in the ABI's edge-order view.
static int read_field_impl(gsim_handle* h, const FieldRef& r, void* dst)
{
    hipError_t e = hipSuccess;
    if (r.kind == FK_RAW) {
        e = hipMemcpyAsync(dst, r.ptr, r.bytes, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        return hip_check(h, e, "gsim_read_field");
    }
    void* tmp = nullptr;
    e = hipMalloc(&tmp, std::max<size_t>(r.bytes, 8));
    if (e != hipSuccess) return hip_check(h, e, "gsim_read_field scratch");
    const int64_t E = h->e;
    const int32_t T = std::max(1, h->t);
    const int64_t total = (int64_t)(r.bytes / (size_t)r.elem);
    const int g = grid_for(total);
    const uint32_t* rev = r.kind == FK_TRECORD ? h->d_rev : nullptr;
    if (r.kind == FK_RECORD && r.elem == 8)
        hipLaunchKernelGGL(k_gather_rev<uint64_t>, dim3(g), dim3(256), 0, h->stream, (const uint64_t*)r.ptr,
                           (uint64_t*)tmp, (const uint32_t*)h->d_rev, E, total);
    else if (r.kind == FK_RECORD || r.kind == FK_ESTATE)
        hipLaunchKernelGGL(k_gather_rev<uint8_t>, dim3(g), dim3(256), 0, h->stream, (const uint8_t*)r.ptr,
                           (uint8_t*)tmp, (const uint32_t*)h->d_rev, E, total);
    else if ((r.kind == FK_TRECORD || r.kind == FK_TEDGE) && r.elem == 8)
        hipLaunchKernelGGL(k_view_read<uint64_t>, dim3(g), dim3(256), 0, h->stream, (const uint64_t*)r.ptr,
                           (uint64_t*)tmp, rev, (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask, E, T, h->S,
                           total);
    else if (r.kind == FK_TRECORD || r.kind == FK_TEDGE)
        hipLaunchKernelGGL(k_view_read<uint8_t>, dim3(g), dim3(256), 0, h->stream, (const uint8_t*)r.ptr,
                           (uint8_t*)tmp, rev, (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask, E, T, h->S,
                           total);
    else
        hipLaunchKernelGGL(k_tflags_compose, dim3(g), dim3(256), 0, h->stream, (const uint8_t*)h->d_tflags,
                           (const uint8_t*)h->d_mflags, (uint8_t*)tmp, (const uint32_t*)h->d_rev,
                           (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask, E, total);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(dst, tmp, r.bytes, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    (void)hipFree(tmp);
    return hip_check(h, e, "gsim_read_field");
}

// The slots a topic-array view written through the ABI needs (its non-zero
// entries), then grow the masks to cover them (ensure_slots).
static int view_slots(gsim_handle* h, const FieldRef& r, const void* dview)
{
    if (!h->d_smask) return GSIM_OK;                      // dense: every topic has its plane
    const int64_t E = h->e;
    const int32_t T = std::max(1, h->t);
    const int64_t total = (int64_t)(r.bytes / (size_t)r.elem);
    unsigned long long* need = nullptr;
    hipError_t e = hipMalloc((void**)&need, sizeof(uint64_t) * (size_t)std::max<int64_t>(h->n, 1));
    if (e == hipSuccess) e = hipMemsetAsync(need, 0, sizeof(uint64_t) * (size_t)h->n, h->stream);
    const uint32_t* rev = h->d_rev;
    const int g = grid_for(total);
    if (e == hipSuccess) {
        if (r.elem == 8)
            hipLaunchKernelGGL(k_view_need<uint64_t>, dim3(g), dim3(256), 0, h->stream, (const uint64_t*)dview, rev,
                               (const uint32_t*)h->d_owner, E, T, total, need);
        else
            hipLaunchKernelGGL(k_view_need<uint8_t>, dim3(g), dim3(256), 0, h->stream, (const uint8_t*)dview, rev,
                               (const uint32_t*)h->d_owner, E, T, total, need);
        e = hipGetLastError();
    }
    std::vector<uint64_t> host((size_t)h->n);
    if (e == hipSuccess) e = hipMemcpyAsync(host.data(), need, sizeof(uint64_t) * (size_t)h->n, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (need) (void)hipFree(need);
    if (e != hipSuccess) return hip_check(h, e, "slot needs");
    return ensure_slots(h, host.data());
}

// Install a field given in the ABI's edge-order view.
static int write_field_impl(gsim_handle* h, int32_t f, const FieldRef& r0, const void* src)
{
    hipError_t e = hipSuccess;
    if (r0.kind == FK_RAW) {
        e = hipMemcpyAsync(r0.ptr, src, r0.bytes, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        return hip_check(h, e, "gsim_write_field");
    }
    void* tmp = nullptr;
    e = hipMalloc(&tmp, std::max<size_t>(r0.bytes, 8));
    if (e != hipSuccess) return hip_check(h, e, "gsim_write_field scratch");
    e = hipMemcpyAsync(tmp, src, r0.bytes, hipMemcpyHostToDevice, h->stream);
    FieldRef r = r0;
    if (e == hipSuccess && (r.kind == FK_TRECORD || r.kind == FK_TEDGE || r.kind == FK_TFLAGS)) {
        const int rc = view_slots(h, r, tmp);
        if (rc) { (void)hipFree(tmp); return rc; }
        field_ref(h, f, &r);      // the arrays may have moved (re-laid out for new slots)
    }
    const int64_t E = h->e;
    const int32_t T = std::max(1, h->t);
    const int64_t total = (int64_t)(r.bytes / (size_t)r.elem);
    const int g = grid_for(total);
    const uint32_t* rev = r.kind == FK_TRECORD ? h->d_rev : nullptr;
    if (e == hipSuccess) {
        if (r.kind == FK_RECORD && r.elem == 8)
            hipLaunchKernelGGL(k_gather_rev<uint64_t>, dim3(g), dim3(256), 0, h->stream, (const uint64_t*)tmp,
                               (uint64_t*)r.ptr, (const uint32_t*)h->d_rev, E, total);
        else if (r.kind == FK_RECORD)
            hipLaunchKernelGGL(k_gather_rev<uint8_t>, dim3(g), dim3(256), 0, h->stream, (const uint8_t*)tmp,
                               (uint8_t*)r.ptr, (const uint32_t*)h->d_rev, E, total);
        else if (r.kind == FK_ESTATE)
            hipLaunchKernelGGL(k_estate_split, dim3(g), dim3(256), 0, h->stream, (const uint8_t*)tmp,
                               h->d_estate, h->d_rstate, (const uint32_t*)h->d_rev, E);
        else if ((r.kind == FK_TRECORD || r.kind == FK_TEDGE) && r.elem == 8)
            hipLaunchKernelGGL(k_view_write<uint64_t>, dim3(g), dim3(256), 0, h->stream, (const uint64_t*)tmp,
                               (uint64_t*)r.ptr, rev, (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask, E, T,
                               h->S, total);
        else if (r.kind == FK_TRECORD || r.kind == FK_TEDGE)
            hipLaunchKernelGGL(k_view_write<uint8_t>, dim3(g), dim3(256), 0, h->stream, (const uint8_t*)tmp,
                               (uint8_t*)r.ptr, rev, (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask, E, T,
                               h->S, total);
        else
            hipLaunchKernelGGL(k_tflags_split, dim3(grid_for((int64_t)T * E)), dim3(256), 0, h->stream,
                               (const uint8_t*)tmp, h->d_tflags, h->d_mflags, (const uint32_t*)h->d_rev,
                               (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask, E, (int64_t)T * E);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    (void)hipFree(tmp);
    return hip_check(h, e, "gsim_write_field");
}

#define GSIM_ENTER(h)                                                     \
    do {                                                                  \
        if (!(h)) return GSIM_EINVAL;                                     \
        hipError_t _e = hipSetDevice((h)->device);                        \
        if (_e != hipSuccess) return hip_check((h), _e, "hipSetDevice");  \
    } while (0)

#define GSIM_NEED_GRAPH(h)                                                \
    do {                                                                  \
        if ((h)->e == 0 && (h)->n == 0) {                                 \
            (h)->err = "no graph loaded (call gsim_load_graph first)";    \
            return GSIM_ESTATE;                                           \
        }                                                                 \
    } while (0)

extern "C" {

static int create_impl(const gsim_peer_score_params* params, const gsim_topic_score_params* topics,
                       int32_t n_topics, const gsim_thresholds* thresholds, const gsim_gossipsub_params* gossip,
                       int32_t device, gsim_handle** out, char* err, size_t errlen, bool validate)
{
    if (!out) return GSIM_EINVAL;
    *out = nullptr;
    auto fail = [&](int rc, const std::string& m) {
        if (err && errlen) std::snprintf(err, errlen, "%s", m.c_str());
        return rc;
    };
    if (!params || !thresholds || !gossip || (n_topics > 0 && !topics))
        return fail(GSIM_EINVAL, "null parameter block");
    if (n_topics < 0 || n_topics > GSIM_MAX_TOPICS) return fail(GSIM_ERANGE, "n_topics must be in [0, 64]");
    char buf[512] = {0};
    if (validate && gsim_validate_peer_params(params, topics, n_topics, buf, sizeof buf))
        return fail(GSIM_EINVAL, buf);
    if (validate && gsim_validate_thresholds(thresholds, buf, sizeof buf)) return fail(GSIM_EINVAL, buf);
    if (gossip->history_gossip > gossip->history_length) {
        std::snprintf(buf, sizeof buf,
                      "invalid parameters for message cache; gossip slots (%d) cannot be larger than history slots (%d)",
                      gossip->history_gossip, gossip->history_length);
        return fail(GSIM_EINVAL, buf);
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(GSIM_EDEVICE, "no HIP device available (the engine has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(GSIM_EINVAL, "device ordinal out of range");
    if (hipSetDevice(device) != hipSuccess) return fail(GSIM_EDEVICE, "hipSetDevice failed");

    gsim_handle* h = new gsim_handle();
    h->device = device;
    h->validate = validate;
    h->pp = *params;
    h->th = *thresholds;
    h->gp = *gossip;
    h->tp.assign(topics, topics + n_topics);
    h->t = n_topics;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return fail(GSIM_EDEVICE, "hipStreamCreate failed");
    }
    for (auto& ev : h->ev) (void)hipEventCreate(&ev);
    if (dalloc(h, &h->d_tp, std::max(1, n_topics)) || dalloc(h, &h->d_flags, 16)) {
        std::string m = h->err;
        gsim_destroy(h);
        return fail(GSIM_ENOMEM, m);
    }
    (void)stream_fill(h, h->d_flags, 0, 16 * sizeof(int32_t));
    h->d_inv_live = reinterpret_cast<uint32_t*>(h->d_flags + 8);
    (void)stream_fill(h, h->d_inv_live, 1, 2 * sizeof(uint32_t));
    if (n_topics > 0)
        (void)stream_copy(h, h->d_tp, topics, sizeof(gsim_topic_score_params) * (size_t)n_topics, hipMemcpyHostToDevice);
    *out = h;
    return GSIM_OK;
}

int gsim_create(const gsim_peer_score_params* params, const gsim_topic_score_params* topics, int32_t n_topics,
                const gsim_thresholds* thresholds, const gsim_gossipsub_params* gossip, int32_t device,
                gsim_handle** out, char* err, size_t errlen)
{
    return create_impl(params, topics, n_topics, thresholds, gossip, device, out, err, errlen, true);
}

int gsim_create_unvalidated(const gsim_peer_score_params* params, const gsim_topic_score_params* topics,
                            int32_t n_topics, const gsim_thresholds* thresholds,
                            const gsim_gossipsub_params* gossip, int32_t device, gsim_handle** out, char* err,
                            size_t errlen)
{
    return create_impl(params, topics, n_topics, thresholds, gossip, device, out, err, errlen, false);
}

int gsim_destroy(gsim_handle* h)
{
    if (!h) return GSIM_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    free_graph(h);
    free_extra(h);
    free_gater(h);
    free_deliver(h);
    trace_release(h);
    dfree(h->d_tp);
    dfree(h->d_flags);
    for (auto& ev : h->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : h->prof_pool) (void)hipEventDestroy(ev);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return GSIM_OK;
}

const char* gsim_last_error(const gsim_handle* h) { return h ? h->err.c_str() : "null handle"; }

int gsim_load_graph(gsim_handle* h, int64_t n, const uint32_t* row_ptr, const uint32_t* col,
                    const uint8_t* outbound, const uint64_t* subs, const uint32_t* ip_ptr, const uint32_t* ip_ids,
                    uint32_t n_ips)
{
    GSIM_ENTER(h);
    if (n <= 0 || !row_ptr || !col) { h->err = "empty graph"; return GSIM_EINVAL; }
    if (n >= (int64_t)UINT32_MAX) { h->err = "too many peers"; return GSIM_ERANGE; }
    const int64_t E = row_ptr[n];
    if (row_ptr[0] != 0) { h->err = "row_ptr[0] must be 0"; return GSIM_EINVAL; }
    // validate the CSR and derive reverse edges / owners on the host
    std::vector<uint32_t> rev((size_t)E), owner((size_t)E);
    for (int64_t i = 0; i < n; ++i) {
        if (row_ptr[i + 1] < row_ptr[i]) { h->err = "row_ptr not monotone"; return GSIM_EINVAL; }
        for (uint32_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
            owner[e] = (uint32_t)i;
            if (col[e] >= (uint64_t)n) { h->err = "col index out of range"; return GSIM_EINVAL; }
            if (col[e] == (uint32_t)i) { h->err = "self loop"; return GSIM_EINVAL; }
            if (e > row_ptr[i] && col[e] <= col[e - 1]) { h->err = "rows must be sorted, no duplicates"; return GSIM_EINVAL; }
        }
    }
    for (int64_t i = 0; i < n; ++i) {
        for (uint32_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
            const uint32_t j = col[e];
            const uint32_t* b = col + row_ptr[j];
            const uint32_t* en = col + row_ptr[j + 1];
            const uint32_t* p = std::lower_bound(b, en, (uint32_t)i);
            if (p == en || *p != (uint32_t)i) { h->err = "graph is not symmetric"; return GSIM_EINVAL; }
            rev[e] = (uint32_t)(p - col);
        }
    }
    if (ip_ptr) {
        if (ip_ptr[0] != 0) { h->err = "ip_ptr[0] must be 0"; return GSIM_EINVAL; }
        if (n_ips > kIpNone) { h->err = "too many IP ids"; return GSIM_EINVAL; }   // ids stay below the P6 key sentinels
        for (int64_t i = 0; i < n; ++i)
            if (ip_ptr[i + 1] < ip_ptr[i]) { h->err = "ip_ptr not monotone"; return GSIM_EINVAL; }
        for (uint32_t q = 0; q < ip_ptr[n]; ++q)
            if (ip_ids[q] >= n_ips) { h->err = "ip id out of range"; return GSIM_EINVAL; }
    }
    if (subs && h->t < 64) {
        const uint64_t mask = h->t == 0 ? 0 : ((1ull << h->t) - 1);
        for (int64_t i = 0; i < n; ++i)
            if (subs[i] & ~mask) { h->err = "subscription bit beyond n_topics"; return GSIM_EINVAL; }
    }

    (void)hipStreamSynchronize(h->stream);
    free_graph(h);
    free_extra(h);
    free_gater(h);
    free_deliver(h);
    trace_release(h);
    h->n = n;
    h->e = E;
    h->n_ips = n_ips;
    // topic slots: the announced topics of every peer; all of
    // them when every peer joined every topic (or none announced any: a
    // caller without subscriptions gets the dense layout)
    const uint64_t tmask_all = h->t >= 64 ? ~0ull : ((1ull << h->t) - 1);
    bool dense_slots = !subs;
    if (subs) {
        bool all = true;
        for (int64_t i = 0; all && i < n; ++i) all = (subs[i] & tmask_all) == tmask_all;
        dense_slots = all;
    }
    h->S = std::max(1, h->t);
    if (!dense_slots) {
        h->smask.assign(subs, subs + n);
        int32_t S = 1;
        for (int64_t i = 0; i < n; ++i) S = std::max(S, __builtin_popcountll(h->smask[(size_t)i]));
        h->S = S;
    }
    const int64_t ET = E * (int64_t)h->S;
    const int64_t nip = ip_ptr ? ip_ptr[n] : 0;
    int rc = GSIM_OK;
    rc = rc ? rc : dalloc(h, &h->d_row_ptr, n + 1);
    rc = rc ? rc : dalloc(h, &h->d_col, E);
    rc = rc ? rc : dalloc(h, &h->d_rev, E);
    rc = rc ? rc : dalloc(h, &h->d_owner, E);
    rc = rc ? rc : dalloc(h, &h->d_sub, n);
    rc = rc ? rc : dalloc(h, &h->d_outbound, E);
    rc = rc ? rc : dalloc(h, &h->d_direct, E);
    rc = rc ? rc : dalloc(h, &h->d_ip_ptr, n + 1);
    rc = rc ? rc : dalloc(h, &h->d_ip_ids, nip);
    rc = rc ? rc : dalloc(h, &h->d_ip_white, (int64_t)n_ips);
    rc = rc ? rc : dalloc(h, &h->d_p5, n);
    rc = rc ? rc : dalloc(h, &h->d_p6row, n);
    rc = rc ? rc : dalloc(h, &h->d_first, ET);
    rc = rc ? rc : dalloc(h, &h->d_meshd, ET);
    rc = rc ? rc : dalloc(h, &h->d_fail, ET);
    rc = rc ? rc : dalloc(h, &h->d_invalid, ET);
    rc = rc ? rc : dalloc(h, &h->d_graft, ET);
    rc = rc ? rc : dalloc(h, &h->d_mtime, ET);
    rc = rc ? rc : dalloc(h, &h->d_tflags, ET);
    rc = rc ? rc : dalloc(h, &h->d_mflags, ET);
    rc = rc ? rc : dalloc(h, &h->d_backoff, ET);
    rc = rc ? rc : dalloc(h, &h->d_rstate, E);
    rc = rc ? rc : dalloc(h, &h->d_dstate, E);
    rc = rc ? rc : dalloc(h, &h->d_pen, E);
    rc = rc ? rc : dalloc(h, &h->d_mcnt, ET);
    rc = rc ? rc : dalloc(h, &h->d_bp, E);
    rc = rc ? rc : dalloc(h, &h->d_estate, E);
    rc = rc ? rc : dalloc(h, &h->d_expire, E);
    rc = rc ? rc : dalloc(h, &h->d_p6, E);
    rc = rc ? rc : dalloc(h, &h->d_score, E);
    if (!dense_slots) rc = rc ? rc : dalloc(h, &h->d_smask, n);
    if (rc) { std::string m = h->err; free_graph(h); h->err = m; return rc; }

    hipStream_t s = h->stream;
    hipError_t he = hipSuccess;
    auto up = [&](void* d, const void* src, size_t bytes) {
        if (he == hipSuccess && bytes) he = hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, s);
    };
    auto zero = [&](void* d, size_t bytes) {
        if (he == hipSuccess && bytes) he = hipMemsetAsync(d, 0, bytes, s);
    };
    up(h->d_row_ptr, row_ptr, sizeof(uint32_t) * (size_t)(n + 1));
    up(h->d_col, col, sizeof(uint32_t) * (size_t)E);
    up(h->d_rev, rev.data(), sizeof(uint32_t) * (size_t)E);
    up(h->d_owner, owner.data(), sizeof(uint32_t) * (size_t)E);
    if (subs) up(h->d_sub, subs, sizeof(uint64_t) * (size_t)n); else zero(h->d_sub, sizeof(uint64_t) * (size_t)n);
    if (!dense_slots) up(h->d_smask, h->smask.data(), sizeof(uint64_t) * (size_t)n);
    {
        // every peer joined every topic: the score pass has nothing to skip
        const uint64_t tmask = h->t >= 64 ? ~0ull : ((1ull << h->t) - 1);
        bool all = subs != nullptr;
        for (int64_t i = 0; all && i < n; ++i) all = (subs[i] & tmask) == tmask;
        h->all_joined = all;
        h->topic_subs.assign((size_t)std::max(1, h->t), 0);
        for (int64_t i = 0; subs && i < n; ++i)
            for (uint64_t b = subs[i] & tmask; b; b &= b - 1) h->topic_subs[__builtin_ctzll(b)]++;
    }
    if (outbound) up(h->d_outbound, outbound, (size_t)E); else zero(h->d_outbound, (size_t)E);
    zero(h->d_direct, (size_t)E);
    h->ip_shared = ips_shared(n, ip_ptr, ip_ids, n_ips);
    if (ip_ptr) {
        up(h->d_ip_ptr, ip_ptr, sizeof(uint32_t) * (size_t)(n + 1));
        up(h->d_ip_ids, ip_ids, sizeof(uint32_t) * (size_t)nip);
    } else {
        zero(h->d_ip_ptr, sizeof(uint32_t) * (size_t)(n + 1));
    }
    zero(h->d_ip_white, (size_t)std::max<uint32_t>(n_ips, 1));
    zero(h->d_p5, sizeof(double) * (size_t)n);
    zero(h->d_first, sizeof(double) * (size_t)ET);
    zero(h->d_meshd, sizeof(double) * (size_t)ET);
    zero(h->d_fail, sizeof(double) * (size_t)ET);
    zero(h->d_invalid, sizeof(double) * (size_t)ET);
    zero(h->d_graft, sizeof(int64_t) * (size_t)ET);
    zero(h->d_mtime, sizeof(int64_t) * (size_t)ET);
    zero(h->d_tflags, (size_t)ET);
    zero(h->d_mflags, (size_t)ET);
    zero(h->d_mcnt, (size_t)ET);
    zero(h->d_pen, (size_t)E);
    zero(h->d_backoff, sizeof(int64_t) * (size_t)ET);
    zero(h->d_bp, sizeof(double) * (size_t)E);
    zero(h->d_expire, sizeof(int64_t) * (size_t)E);
    zero(h->d_p6, sizeof(double) * (size_t)E);
    zero(h->d_score, sizeof(double) * (size_t)E);
    if (he != hipSuccess) return hip_check(h, he, "graph upload");
    // AddPeer for every connection (score.go:595-609): tracked + connected
    hipLaunchKernelGGL(k_fill_u8, dim3(grid_for(E)), dim3(256), 0, s, h->d_estate, E,
                       (uint8_t)(GSIM_ES_TRACKED | GSIM_ES_CONNECTED));
    hipLaunchKernelGGL(k_fill_u8, dim3(grid_for(E)), dim3(256), 0, s, h->d_rstate, E, (uint8_t)GSIM_ES_CONNECTED);
    hipLaunchKernelGGL(k_fill_u8, dim3(grid_for(n)), dim3(256), 0, s, h->d_p6row, n, (uint8_t)0);
    h->score_version++;
    h->mesh_version++;
    h->has_white = false;
    h->p6_dirty = true; h->p6_rows_only = false;
    h->maybe_retained = false;
    h->mcnt_dirty = false;
    h->mt_lazy = false;
    h->unjoined_zero = true;     // all state zero
    int rc2 = alloc_extra(h);
    if (rc2) return rc2;
    he = hipStreamSynchronize(s);
    return hip_check(h, he, "gsim_load_graph");
}

int gsim_set_app_score(gsim_handle* h, const double* p5)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    if (!p5) return GSIM_EINVAL;
    hipError_t e = hipMemcpyAsync(h->d_p5, p5, sizeof(double) * (size_t)h->n, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return hip_check(h, e, "gsim_set_app_score");
}

int gsim_set_direct_peers(gsim_handle* h, const uint8_t* direct)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    hipError_t e = direct ? hipMemcpyAsync(h->d_direct, direct, (size_t)h->e, hipMemcpyHostToDevice, h->stream)
                          : hipMemsetAsync(h->d_direct, 0, (size_t)h->e, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    h->score_version++;
    h->mesh_version++;          // AcceptFrom and the send sets read the flags through the delivery state
    return hip_check(h, e, "gsim_set_direct_peers");
}

int gsim_set_ips(gsim_handle* h, const uint32_t* ip_ptr, const uint32_t* ip_ids, uint32_t n_ips)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    if (!ip_ptr || ip_ptr[0] != 0) { h->err = "ip_ptr[0] must be 0"; return GSIM_EINVAL; }
    if (n_ips > kIpNone) { h->err = "too many IP ids"; return GSIM_EINVAL; }
    if (h->gt) {
        // the peer gater's per-IP groups are built by gsim_set_peer_gater from the IPs then
        h->err = "gsim_set_ips with the peer gater on: set the IPs before gsim_set_peer_gater";
        return GSIM_ESTATE;
    }
    const int64_t n = h->n;
    for (int64_t i = 0; i < n; ++i)
        if (ip_ptr[i + 1] < ip_ptr[i]) { h->err = "ip_ptr not monotone"; return GSIM_EINVAL; }
    const int64_t nip = ip_ptr[n];
    if (nip > 0 && !ip_ids) { h->err = "ip_ids missing"; return GSIM_EINVAL; }
    for (int64_t q = 0; q < nip; ++q)
        if (ip_ids[q] >= n_ips) { h->err = "ip id out of range"; return GSIM_EINVAL; }
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_set_ips");
    dfree(h->d_ip_ids);
    int rc = dalloc(h, &h->d_ip_ids, nip);
    if (!rc && n_ips != h->n_ips) {
        dfree(h->d_ip_white);
        rc = dalloc(h, &h->d_ip_white, (int64_t)n_ips);
        h->has_white = false;
        if (!rc) e = hipMemsetAsync(h->d_ip_white, 0, std::max<size_t>(n_ips, 1), h->stream);
    }
    if (rc) return rc;
    h->n_ips = n_ips;
    if (e == hipSuccess) e = hipMemcpyAsync(h->d_ip_ptr, ip_ptr, sizeof(uint32_t) * (size_t)(n + 1), hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess && nip) e = hipMemcpyAsync(h->d_ip_ids, ip_ids, sizeof(uint32_t) * (size_t)nip, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    h->p6_dirty = true; h->p6_rows_only = false;
    h->ip_shared = ips_shared(n, ip_ptr, ip_ids, n_ips);
    return hip_check(h, e, "gsim_set_ips");
}

int gsim_set_ip_whitelist(gsim_handle* h, const uint8_t* white)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    hipError_t e = hipSuccess;
    if (white && h->n_ips) {
        e = hipMemcpyAsync(h->d_ip_white, white, (size_t)h->n_ips, hipMemcpyHostToDevice, h->stream);
        h->has_white = true;
    } else {
        h->has_white = false;
    }
    h->p6_dirty = true; h->p6_rows_only = false;
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return hip_check(h, e, "gsim_set_ip_whitelist");
}

int gsim_set_topic_params(gsim_handle* h, int32_t t, const gsim_topic_score_params* p)
{
    GSIM_ENTER(h);
    if (!p || t < 0 || t >= h->t) { h->err = "topic index out of range"; return GSIM_EINVAL; }
    char buf[256] = {0};
    if (h->validate && p->scored && gsim_validate_topic_params(p, buf, sizeof buf)) { h->err = buf; return GSIM_EINVAL; }
    int rcf = deliver_flush(h);
    if (!rcf) rcf = materialize_mcnt(h);   // pending increments saw the old cap
    if (!rcf) rcf = materialize_mtime(h, true);   // the records the refresh rewrites may change
    if (rcf) return rcf;
    const gsim_topic_score_params old = h->tp[t];
    h->tp[t] = *p;
    hipError_t e = hipMemcpyAsync(h->d_tp + t, p, sizeof(*p), hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = inv_mark_all(h);   // a topic now scored: its records are read again
    if (e != hipSuccess) return hip_check(h, e, "gsim_set_topic_params");
    if (old.scored && h->e > 0) {
        const int df = p->first_message_deliveries_cap < old.first_message_deliveries_cap;
        const int dm = p->mesh_message_deliveries_cap < old.mesh_message_deliveries_cap;
        if (df || dm) {
            hipLaunchKernelGGL(k_recap, dim3(grid_for(h->e)), dim3(256), 0, h->stream, h->e, h->d_estate,
                               (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask, t, h->d_first,
                               h->d_meshd, p->first_message_deliveries_cap, p->mesh_message_deliveries_cap, df, dm);
            e = hipGetLastError();
        }
    }
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return hip_check(h, e, "gsim_set_topic_params");
}

int gsim_refresh_scores(gsim_handle* h, int64_t now)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    return launch_refresh_scores(h, now);
}

int gsim_compute_scores(gsim_handle* h)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    return launch_compute_scores(h);
}

int gsim_compute_ip_colocation(gsim_handle* h)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    return launch_ip_colocation(h);
}

int gsim_fill_synthetic(gsim_handle* h, uint64_t seed, int64_t now, double p_mesh)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    int rcf = deliver_flush(h);
    if (!rcf) rcf = materialize_mcnt(h);
    if (rcf) return rcf;
    ScoreArgs a = make_score_args(h, now);
    hipLaunchKernelGGL(k_fill_synthetic, dim3(grid_for(h->e)), dim3(256), 0, h->stream, a, seed, p_mesh);
    (void)inv_mark_all(h);
    h->mt_lazy = false;          // the fill stores meshTime
    h->p6_dirty = true; h->p6_rows_only = false;
    h->score_version++;
    h->mesh_version++;
    h->maybe_retained = false;
    h->unjoined_zero = true;     // the fill leaves records of unshared topics zero
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return hip_check(h, e, "gsim_fill_synthetic");
}

int gsim_set_kernel_variant(gsim_handle* h, int32_t which, int32_t variant)
{
    if (!h) return GSIM_EINVAL;
    if (which == 2) {           // delivery: 3 = topic-major k_send_tm (the only kernel; the peer-major one is gone)
        if (variant != 3) { h->err = "unknown delivery kernel variant (3: topic-major)"; return GSIM_EINVAL; }
        return GSIM_OK;
    }
    if (which == 3) {           // k_ihave lane group: 0 = by row lengths, else 8 / 16 / 32 / 64
        if (variant != 0 && variant != 8 && variant != 16 && variant != 32 && variant != 64) {
            h->err = "unknown IHAVE lane width (0, 8, 16, 32 or 64)";
            return GSIM_EINVAL;
        }
        h->ihave_w = variant;
        return GSIM_OK;
    }
    if (which == 9) {           // sparse rounds: 0 = the list-driven send where the configuration allows, 1 = the scan
        if (variant < 0 || variant > 1) { h->err = "unknown send driver (0 or 1)"; return GSIM_EINVAL; }
        h->flist_off = variant == 1;
        return GSIM_OK;
    }
    if (which == 8) {           // k_xbits_deliver: 0 = batched copies where the configuration allows, 1 = one at a time
        if (variant < 0 || variant > 1) { h->err = "unknown bit-apply variant (0 or 1)"; return GSIM_EINVAL; }
        h->xb_generic = variant == 1;
        return GSIM_OK;
    }
    if (which == 6) {           // topic-major blocks: 0 = shared out by subscribers, 1 = the same per topic,
                                // >= 64: shared out by subscribers, this many in all
        if (variant < 0 || (variant > 1 && variant < 64)) { h->err = "unknown block share (0, 1 or >= 64)"; return GSIM_EINVAL; }
        h->tm_uniform = variant == 1;
        h->tm_budget = variant >= 64 ? variant : 0;
        if (h->dl) deliver_blocks_changed(h);
        return GSIM_OK;
    }
    h->err = "unknown kernel variant class";
    return GSIM_EINVAL;
}

int gsim_census(gsim_handle* h, int64_t* out8)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    if (!out8) return GSIM_EINVAL;
    int rcf = deliver_flush(h);
    if (rcf) return rcf;
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc((void**)&d, 8 * sizeof(unsigned long long));
    if (e != hipSuccess) return hip_check(h, e, "hipMalloc census");
    e = hipMemsetAsync(d, 0, 8 * sizeof(unsigned long long), h->stream);
    ScoreArgs a = make_score_args(h, 0);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_census, dim3(grid_for(h->e, 256, 4096)), dim3(256), 0, h->stream, a, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out8, d, 8 * sizeof(int64_t), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    (void)hipFree(d);
    return hip_check(h, e, "gsim_census");
}

int gsim_read_scores(gsim_handle* h, double* out)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    if (!out) return GSIM_EINVAL;
    FieldRef r;
    field_ref(h, GSIM_F_SCORE, &r);
    return read_field_impl(h, r, out);
}

int gsim_field_bytes(gsim_handle* h, int32_t f, size_t* out)
{
    if (!h || !out) return GSIM_EINVAL;
    FieldRef r;
    if (!field_ref(h, f, &r)) { h->err = "unknown field"; return GSIM_EINVAL; }
    *out = r.bytes;
    return GSIM_OK;
}

int gsim_read_field(gsim_handle* h, int32_t f, void* dst, size_t bytes)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    FieldRef r;
    if (!field_ref(h, f, &r)) { h->err = "unknown field"; return GSIM_EINVAL; }
    if (bytes != r.bytes || !dst) { h->err = "field size mismatch"; return GSIM_EINVAL; }
    if (r.kind == FK_SEEN) return deliver_read_seen(h, dst);
    int rc = deliver_flush(h);
    if (!rc) rc = materialize_mcnt(h);
    if (!rc && f == GSIM_F_MESH_TIME) rc = materialize_mtime(h, false);
    if (rc) return rc;
    return read_field_impl(h, r, dst);
}

int gsim_write_field(gsim_handle* h, int32_t f, const void* src, size_t bytes)
{
    GSIM_ENTER(h);
    GSIM_NEED_GRAPH(h);
    FieldRef r;
    if (!field_ref(h, f, &r)) { h->err = "unknown field"; return GSIM_EINVAL; }
    if (bytes != r.bytes || !src) { h->err = "field size mismatch"; return GSIM_EINVAL; }
    if (r.kind == FK_SEEN) { h->err = "the seen-set is read-only"; return GSIM_EINVAL; }
    int rc = deliver_flush(h);
    if (!rc) rc = materialize_mcnt(h);
    if (!rc) rc = materialize_mtime(h, true);   // arbitrary state: meshTime is stored again
    // fanout state lives in the publisher's topic slots
    if (!rc && f == GSIM_F_FANOUT_TOPICS) rc = ensure_slots(h, (const uint64_t*)src);
    if (rc) return rc;
    rc = write_field_impl(h, f, r, src);
    h->unjoined_zero = false;    // arbitrary state: no record may be skipped
    if (!rc) rc = hip_check(h, inv_mark_all(h), "gsim_write_field");
    if (!rc) rc = extra_field_written(h, f);
    if (f == GSIM_F_ESTATE) { h->p6_dirty = true; h->p6_rows_only = false; h->maybe_retained = true; h->score_version++;
    h->mesh_version++; }
    if (f == GSIM_F_SCORE) h->score_version++;
    h->mesh_version++;          // router flags may have changed (delivery's mesh masks)
    h->mesh_version++;
    return rc;
}

int gsim_event_record(gsim_handle* h, int32_t slot)
{
    GSIM_ENTER(h);
    if (slot < 0 || slot >= kEvents) return GSIM_EINVAL;
    return hip_check(h, hipEventRecord(h->ev[slot], h->stream), "hipEventRecord");
}

int gsim_event_elapsed(gsim_handle* h, int32_t from, int32_t to, float* ms)
{
    GSIM_ENTER(h);
    if (from < 0 || from >= kEvents || to < 0 || to >= kEvents || !ms) return GSIM_EINVAL;
    hipError_t e = hipEventSynchronize(h->ev[to]);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, h->ev[from], h->ev[to]);
    return hip_check(h, e, "hipEventElapsedTime");
}

int gsim_synchronize(gsim_handle* h)
{
    GSIM_ENTER(h);
    return hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
}

int gsim_profile(gsim_handle* h, int32_t enable)
{
    GSIM_ENTER(h);
    hipError_t e = hipStreamSynchronize(h->stream);
    h->prof_on = enable != 0;
    h->prof_used = 0;
    h->prof_lost = false;
    h->prof_marks.clear();
    return hip_check(h, e, "gsim_profile");
}

int gsim_profile_read(gsim_handle* h, double* ms, int64_t* launches, int32_t n)
{
    GSIM_ENTER(h);
    if (n < 0 || (n > 0 && (!ms || !launches))) return GSIM_EINVAL;
    for (int32_t c = 0; c < n; ++c) { ms[c] = 0.0; launches[c] = 0; }
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_profile_read");
    for (const auto& m : h->prof_marks) {
        float t = 0.f;
        e = hipEventElapsedTime(&t, h->prof_pool[m.a], h->prof_pool[m.b]);
        if (e != hipSuccess) return hip_check(h, e, "hipEventElapsedTime");
        if (m.cls < n) { ms[m.cls] += t; launches[m.cls] += 1; }
    }
    const bool lost = h->prof_lost;
    h->prof_marks.clear();
    h->prof_used = 0;
    h->prof_lost = false;
    if (lost) { h->err = "profile event pool exhausted; totals are partial"; return GSIM_ERANGE; }
    return GSIM_OK;
}

}  // extern "C"

static int32_t prof_mark(gsim_handle* h)
{
    constexpr size_t kProfMax = 1 << 16;
    if (!h->prof_on) return -1;
    if (h->prof_used == h->prof_pool.size()) {
        hipEvent_t ev = nullptr;
        if (h->prof_pool.size() >= kProfMax || hipEventCreate(&ev) != hipSuccess) {
            h->prof_lost = true;
            return -1;
        }
        h->prof_pool.push_back(ev);
    }
    if (hipEventRecord(h->prof_pool[h->prof_used], h->stream) != hipSuccess) {
        h->prof_lost = true;
        return -1;
    }
    return (int32_t)h->prof_used++;
}

ProfScope::ProfScope(gsim_handle* hh, int32_t c) : h(hh), cls(c), a(prof_mark(hh)) {}

ProfScope::~ProfScope()
{
    if (a < 0) return;
    const int32_t b = prof_mark(h);
    if (b >= 0) h->prof_marks.push_back({cls, (uint32_t)a, (uint32_t)b});
}

bool field_ref(gsim_handle* h, int32_t f, FieldRef* r)
{
    const size_t E = (size_t)h->e, ET = E * (size_t)std::max(1, h->t);
    switch (f) {
    case GSIM_F_FIRST:      *r = {h->d_first, ET * 8, FK_TRECORD, 8}; return true;
    case GSIM_F_MESHD:      *r = {h->d_meshd, ET * 8, FK_TRECORD, 8}; return true;
    case GSIM_F_FAIL:       *r = {h->d_fail, ET * 8, FK_TRECORD, 8}; return true;
    case GSIM_F_INVALID:    *r = {h->d_invalid, ET * 8, FK_TRECORD, 8}; return true;
    case GSIM_F_GRAFT_TIME: *r = {h->d_graft, ET * 8, FK_TRECORD, 8}; return true;
    case GSIM_F_MESH_TIME:  *r = {h->d_mtime, ET * 8, FK_TRECORD, 8}; return true;
    case GSIM_F_TFLAGS:     *r = {h->d_tflags, ET, FK_TFLAGS, 1}; return true;
    case GSIM_F_BP:         *r = {h->d_bp, E * 8, FK_RECORD, 8}; return true;
    case GSIM_F_ESTATE:     *r = {h->d_estate, E, FK_ESTATE, 1}; return true;
    case GSIM_F_EXPIRE:     *r = {h->d_expire, E * 8, FK_RECORD, 8}; return true;
    case GSIM_F_P6:         *r = {h->d_p6, E * 8, FK_RECORD, 8}; return true;
    case GSIM_F_SCORE:      *r = {h->d_score, E * 8, FK_RECORD, 8}; return true;
    case GSIM_F_BACKOFF:    *r = {h->d_backoff, ET * 8, FK_TEDGE, 8}; return true;
    default: return extra_field_ref(h, f, r) || deliver_field_ref(h, f, r);
    }
}
