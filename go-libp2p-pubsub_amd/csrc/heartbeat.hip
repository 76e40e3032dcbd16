// heartbeat.hip — GossipSub heartbeat mesh maintenance and control handling.
//
// gossipsub.go:1345-1606 runs once per node per heartbeat over Go maps.  Here
// one 64-lane wavefront owns one observer: lane l holds the observer's l-th
// connection (its score snapshot, outbound flag, neighbour subscriptions),
// so every per-topic set operation of the reference (mesh size, filtered
// candidate lists, getPeers' shuffle+truncate, the Dhi score sort, the
// opportunistic median) becomes a wave ballot, popcount or keyed
// min-reduction with no memory traffic beyond the row's own records.
// Topics are processed in ascending order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "gsim.h"
#include "gsim_internal.h"
#include "philox.h"

using namespace gsim;

constexpr int kGiantRow = 8192;   // longest row the heartbeat takes (k_heartbeat_hub_g)
// row positions per thread of the heartbeat's hub classes (below)
#ifndef GSIM_HB_HUBV
#define GSIM_HB_HUBV 2
#endif
// classes: rows of 65-128, -256, -512, -1024, -2048, -4096 connections; threads x
// positions per thread cover the class's longest row.  Scheme 1: blocks as wide as
// the row (2 and 4 positions from 1025); 2: two positions per thread up to 1024
// connections; 3: four from 129 to 1024 (≈95 VGPRs per position: 380-410, one wave
// per SIMD, no scratch; 512 x 4 and 512 x 8 would spill 157 / 1373, so the 1025-4096
// classes keep 1024 threads)
#define GSIM_HUB_SCHEME_(s1, s2, s3) (GSIM_HB_HUBV == 1 ? (s1) : GSIM_HB_HUBV == 2 ? (s2) : (s3))
constexpr int kHubB[6] = {GSIM_HUB_SCHEME_(128, 64, 64), GSIM_HUB_SCHEME_(256, 128, 64), GSIM_HUB_SCHEME_(512, 256, 128),
                          GSIM_HUB_SCHEME_(1024, 512, 256), 1024, 1024};
constexpr int kHubVv[6] = {GSIM_HUB_SCHEME_(1, 2, 2), GSIM_HUB_SCHEME_(1, 2, 4), GSIM_HUB_SCHEME_(1, 2, 4),
                           GSIM_HUB_SCHEME_(1, 2, 4), 2, 4};
static_assert(kHubB[0] * kHubVv[0] == 128 && kHubB[1] * kHubVv[1] == 256 && kHubB[2] * kHubVv[2] == 512 &&
              kHubB[3] * kHubVv[3] == 1024 && kHubB[4] * kHubVv[4] == 2048 && kHubB[5] * kHubVv[5] == 4096,
              "a hub class's block covers its longest row");

struct Extra {
    uint8_t* d_ctl = nullptr;   // [2][T][E] control inbox by round parity
    uint64_t* d_cany = nullptr;  // [2][N] per receiver: topics that may hold control (a superset), by parity
    int64_t* d_lastpub = nullptr;      // [N][T] gs.lastpub (ns), 0 = none
    uint64_t* d_fantopics = nullptr;   // [N] bit t: gs.fanout[t] exists
    uint32_t max_degree = 0;
    uint64_t seed = 0x9E3779B97F4A7C15ull;
    // observers by row length for the heartbeat's lane groups: [0, n16) rows
    // of <= 16 connections, then <= 32, then the rest (nullptr: one class)
    uint32_t* d_rows = nullptr;
    int64_t n16 = 0, n32 = 0, n64 = 0;
    int64_t n8 = 0;            // the first n8 rows of [0, n16) hold at most 8 connections (k_heartbeat<8>)
    // hub observers after them: rows of 65..256, 257..1024, then 1025..4096
    // connections (a block of 1024 threads holding 4 row positions each)
    int64_t nh256 = 0, nh1024 = 0, nh4096 = 0;
    int64_t nh2048 = 0;                 // the first rows of the 1025-4096 class, of at most 2048 connections
    int64_t nh128 = 0, nh512 = 0;       // ... of the 65-256 class of at most 128, of the 257-1024 class of at most 512
    // rows of 4097..8192 connections (the reference's heartbeat has no degree
    // bound, gossipsub.go:1386-1557): a block of 1024 threads holding 8 row
    // positions each, whose group state lives in global scratch (d_gscratch:
    // one BlockGroup<1024, 8>::Shared per block, 278 KB -- more than the LDS)
    int64_t nh8192 = 0;
    void* d_gscratch = nullptr;
    int64_t gscratch_blocks = 0;
    // peer exchange (gsim_gossipsub_params.do_px): topics with PX PRUNEs per
    // observer, connection attempts per edge, the GRAFT RPCs that turned PX off
    uint64_t* d_pxo = nullptr;
    uint8_t* d_pxm = nullptr;
    uint8_t* d_nopx = nullptr;
    uint32_t* d_pxc = nullptr;         // [1 + 2E] connections made: count, then (dialer edge, peer edge)
    double* d_pxs = nullptr;           // [E] live scores of PX observers (HbArgs::pxs)
    // Leave's PRUNEs with PX (makePrune(p, topic, doPX, true), gossipsub.go:1118): their
    // lists, one entry per listed peer (the pruner's edge | topic << 32 | listed peer's
    // global id << 38) and the Leave's tick, until the connector (gsim_px_connect)
    // hands them to the pruned peers and the wire encoder has read them
    uint64_t* d_pxl = nullptr;
    uint32_t* d_pxl_tick = nullptr;
    uint32_t* d_pxl_n = nullptr;       // [2] entries, overflow
    int64_t pxl_cap = 0;
};

struct HbArgs {
    int64_t N, E;
    int32_t T;
    const uint32_t *row_ptr, *col, *rev;
    const uint64_t* sub;
    // every peer announced every topic (and no Join / Leave since): a
    // neighbour's subscriptions are the full mask, not a gather of sub[col]
    int32_t sub_all;
    // the refresh's invalidMessageDeliveries flag (engine.hip, inv_mark): 0 =
    // every record's counter is zero, so score_of_record loads no invalid plane
    const uint32_t* inv_live;
    const uint64_t* smask;     // topic slots of each row owner (nullptr: dense; gsim_internal.h)
    const uint8_t* outbound;
    const uint8_t* direct;     // [E] edge order: col[e] is in the observer's gs.direct set
    const uint8_t* estate;
    const double* score;
    const gsim_topic_score_params* tp;
    uint8_t* mflags;    // router mesh bit, edge order [T][E]
    const uint8_t* rstate;   // router connected bit, edge order [E]
    uint8_t* tflags;    // score bits (inMesh, active), record order [T][E]
    int64_t* backoff;
    double *meshd, *fail, *bp;
    uint8_t* mcnt;             // pending meshd increments (k_churn_apply applies the ones it reads)
    int64_t *graft, *mtime;
    int32_t mt_lazy;    // lazy meshTime since the refresh at mt_R (lazy_mtime)
    int64_t mt_R;
    uint8_t* ctl_in;    // inbox this phase reads (round parity)
    uint8_t* ctl_out;   // inbox this phase writes
    uint64_t* cany_in;  // [N] topics with pending control per receiver (ctl_in), cleared when handled
    uint64_t* cany_out; // [N] ... for ctl_out: a sender sets bit t when it writes receiver's entry
    uint64_t tick;
    int64_t now;
    uint64_t seed;
    int32_t D, Dlo, Dhi, Dscore, Dout, opp_peers;
    uint64_t opp_ticks;
    int64_t prune_backoff, graft_flood;
    int64_t unsub_backoff;     // UnsubscribeBackoff (Leave's PRUNE, GSIM_CTL_UNSUB)
    double opp_threshold;
    // emitGossip (gossipsub.go:1711-1775); gossip == false before gsim_msgs_init
    bool gossip;
    const int32_t* lastput;    // [T][N]
    uint8_t* gsel;             // [T][E] sender edge order: emitGossip chose col[e] this heartbeat
    uint8_t* gstate;           // [E] edge order: snapshot score >= gossipThreshold
    double gossip_thr, gossip_factor;
    int32_t dlazy, hist_gossip;
    // live Score(p) for emitGossip (score.go:265-342)
    const double *first, *invalid, *p5, *p6;
    double topic_cap, w5, w6, bp_thr, w7;
    // fanout (gossipsub.go:1011-1028, 1558-1596); router bit GSIM_TF_FANOUT in mflags
    int64_t* lastpub;          // [N][T]
    uint64_t* fan_topics;      // [N]
    double pub_thr;
    int64_t fanout_ttl;
    // sharded network: observers / receivers [olo, ohi) are
    // this shard's; selection keys use global peer ids (gid, nullptr: local = global)
    const uint32_t* gid;
    uint32_t olo, ohi;
    uint64_t* mmask;           // [T][N] delivery's mesh masks (nullptr before gsim_msgs_init)
    uint32_t mlo, mhi;         // ... of edges to [mlo, mhi): a shard's owned peers (pull) or all (push)
    // a shard's control pass: mesh changes of cross edges for the other shards'
    // ghost rows (src | dest << 6 | topic << 12 | flags << 20 | position << 32)
    uint64_t* rdel;
    uint32_t* rdel_n;
    int64_t rdel_cap;
    const uint32_t* xq;
    ShardRanges sr;
    // peer exchange (makePrune doPX, gossipsub.go:1866-1906; pxConnect 893-939)
    int32_t do_px, prune_peers;
    double accept_px;
    uint64_t* pxo;             // [N] topics in which the observer sent a PRUNE with PX
    // sharded: a PRUNE with PX to a ghost goes to the ghost's shard, one entry per
    // listed peer (the cross edge's index there | topic << 32 | listed peer's
    // global id << 38) in per-destination lists [K][pxcap] (pxcnt[K]: overflow)
    uint64_t* pxout;
    uint32_t* pxcnt;
    int64_t pxcap;
    int32_t pxK;
    const uint32_t* xre;       // ShardCtx::d_xre
    const uint8_t* pshard;
    uint8_t* pxm;              // [E] the row's owner tries to connect to col[e]
    uint8_t* nopx;             // [E] a GRAFT of this sender turned PX off for its RPC
    double* pxs;               // [E] the observer's live score of col[e] after its heartbeat (PX observers)
    uint64_t* pxl;             // Leave's PX lists (Extra::d_pxl), their ticks, count
    uint32_t* pxl_tick;
    uint32_t* pxl_n;
    int64_t pxl_cap;
    TraceRef tr;               // gsim_trace_config: tracer.Graft / Prune / AddPeer / RemovePeer
};

namespace {

constexpr int64_t kSecond = 1000000000LL;
constexpr int64_t kBackoffSlack = 2 * kSecond;   // 2*GossipSubHeartbeatInterval (gossipsub.go:1638)
#ifndef GSIM_FLAG_CHUNK
#define GSIM_FLAG_CHUNK 8
#endif
constexpr int kFlagChunk = GSIM_FLAG_CHUNK;      // topics whose flags are loaded together

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// Minimum of a 32-bit value over the 64 lanes with DPP row shifts and row
// broadcasts (VALU data paths, no LDS permute); every lane must be active.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
    const int I = -1;   // 0xFFFFFFFF: identity of min for lanes a shift leaves empty
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x111, 0xF, 0xF, false));   // row_shr:1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x112, 0xF, 0xF, false));   // row_shr:2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x114, 0xF, 0xF, false));   // row_shr:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x118, 0xF, 0xF, false));   // row_shr:8
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x142, 0xA, 0xF, false));   // row_bcast:15
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x143, 0xC, 0xF, false));   // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Minimum over the W-lane group `grp` (W = 32: lanes 0-31 or 32-63; W = 16:
// one 16-lane DPP row; W = 8: half a row -- after the row shifts by 1, 2 and 4,
// lane 7 and lane 15 of a row hold its halves' minima, each read only through
// lanes of its own half).  The row shifts and the row_bcast:15 step read only
// lanes of the same group, so a group may run this while other groups of the
// wave are inactive.
template <int W>
__device__ __forceinline__ uint32_t group_min_u32(uint32_t v, int grp)
{
    if constexpr (W == 64) {
        return wave_min_u32(v);
    } else {
        static_assert(W == 32 || W == 16 || W == 8, "groups of 8, 16, 32 or 64 lanes");
        const int I = -1;
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x111, 0xF, 0xF, false));   // row_shr:1
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x112, 0xF, 0xF, false));   // row_shr:2
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x114, 0xF, 0xF, false));   // row_shr:4
        if constexpr (W == 8) {
            uint32_t r = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)v, 8 * q + 7);
                if (grp == q) r = x;
            }
            return r;
        }
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x118, 0xF, 0xF, false));   // row_shr:8
        if constexpr (W == 32) {
            v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x142, 0xA, 0xF, false));   // row_bcast:15
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
            return grp ? hi : lo;
        } else {
            // lane 15 of each 16-lane row holds the row's minimum
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
            const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
            const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
            const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
            return grp == 0 ? r0 : grp == 1 ? r1 : grp == 2 ? r2 : r3;
        }
    }
}

// The global id of a local peer: selection keys are those of the whole network.
__device__ __forceinline__ uint32_t glob(const HbArgs& a, uint32_t p) { return a.gid ? a.gid[p] : p; }

__device__ __forceinline__ uint64_t hb_key(const HbArgs& a, uint32_t obs, int32_t t, uint32_t purpose, uint32_t col,
                                           uint32_t pos)
{
    return select_key(a.seed, (uint32_t)a.tick, obs, (uint32_t)t, purpose, col, pos);
}

__device__ __forceinline__ uint32_t hb_key_hi(const HbArgs& a, uint32_t obs, int32_t t, uint32_t purpose,
                                              uint32_t col, uint32_t pos)
{
    return (uint32_t)(select_key(a.seed, (uint32_t)a.tick, obs, (uint32_t)t, purpose, col, pos) >> 32);
}

// getPeers (gossipsub.go:1908-1928) restated: among candidate lanes keep the
// `count` with the smallest Philox key (all of them if count <= 0 or fewer).
// A key is (32 random bits, row position); the row position is the lane, so
// each round takes the wave minimum of the random word and breaks ties by
// the lowest lane.
//
// The keys are uniform, so a threshold tau = count/n of the key range already
// selects about `count` lanes with one ballot; the few lanes too many (or too
// few) are then removed largest-first (added smallest-first) by wave
// reductions.  Keys below tau precede every key above it whatever the lane, so
// the result is exactly the `count` smallest (key, lane) pairs.
//
// W-lane groups (W = 32: two observers per wave): every ballot is masked to
// the caller's group `gm`, the lane index keeps breaking ties (the group's
// lanes are in row order), and a group may run this alone.
template <int W = 64>
__device__ bool select_smallest(const HbArgs& a, bool cand, int count, uint32_t obs, int32_t t, uint32_t purpose,
                                uint32_t col, uint32_t pos, uint64_t gm = ~0ull, int grp = 0)
{
    const uint64_t avail = __ballot(cand) & gm;
    const int n = __popcll(avail);
    if (n == 0) return false;
    if (count <= 0 || n <= count) return cand;
    const int lane = threadIdx.x & 63;
    uint32_t hi = 0xFFFFFFFFu;
    if (cand) hi = hb_key_hi(a, obs, t, purpose, col, pos);
    // any threshold gives the same selection; it only sets how many lanes the
    // loops below adjust (fp32: no 64-bit integer division)
    const uint32_t tau = (uint32_t)((float)count / (float)n * 4294967040.0f);
    bool sel = cand && hi < tau;
    int c = __popcll(__ballot(sel) & gm);
    while (c > count) {                 // drop the largest (key, lane) among the selected
        const uint32_t mx = ~group_min_u32<W>(sel ? ~hi : 0xFFFFFFFFu, grp);
        const uint64_t at = __ballot(sel && hi == mx) & gm;
        const int win = 63 - __clzll((long long)at);
        if (lane == win) sel = false;
        --c;
    }
    uint32_t rest = (cand && !sel) ? hi : 0xFFFFFFFFu;
    uint64_t left = __ballot(cand && !sel) & gm;
    while (c < count) {                 // add the smallest (key, lane) among the others
        const uint32_t mn = group_min_u32<W>(rest, grp);
        const int win = __ffsll((long long)(__ballot(rest == mn) & left)) - 1;
        left &= ~(1ull << win);
        if (lane == win) { sel = true; rest = 0xFFFFFFFFu; }
        ++c;
    }
    return sel;
}

// The kernel arguments re-read per topic: every pointer of HbArgs hoisted out
// of the topic loop would otherwise stay live in SGPRs across it, and the
// excess spills to VGPR lanes (v_readlane per use).  The opaque pointer keeps
// the scalar loads (constant address space, K$ hits) inside the loop.
// Only for kernels whose first parameter is the HbArgs (k_heartbeat,
// k_heartbeat_hub): it is read at the start of the kernarg segment.
__device__ __forceinline__ const HbArgs& hb_launder(const HbArgs& a)
{
    return kernarg0(a);        // (the same re-read; debug builds check its argument)
}

// The score bits of one (observer, neighbour, topic) record, loaded on first
// use: Graft/Prune are rare, and the record lives at rev[e] (record order,
// DESIGN.md §2), away from the observer's row.
struct ScoreFlags {
    int64_t ir;          // record index: topic t's slot of the neighbour's row, at rev[e]
    bool ok = false;     // the neighbour holds a slot for t (else the record is absent: zero)
    uint8_t v = 0, v0 = 0;
    bool have = false;
    __device__ void at(uint64_t mj, int32_t t, int64_t E, uint32_t rv)
    {
        ok = slot_has(mj, t);
        ir = slot_idx(mj, t, E, rv);
    }
    __device__ uint8_t& get(const HbArgs& a)
    {
        if (!have) { v = v0 = ok ? a.tflags[ir] : 0; have = true; }
        return v;
    }
    __device__ void store(const HbArgs& a) const
    {
        if (ok && have && v != v0) a.tflags[ir] = v;
    }
};

// peerScore.Graft / Prune on one edge-topic record (score.go:649-691)
__device__ __forceinline__ void stats_graft(const HbArgs& a, bool tracked, bool scored, ScoreFlags& sf)
{
    if (!tracked || !scored || !sf.ok) return;
    uint8_t& fl = sf.get(a);
    fl = (uint8_t)((fl | GSIM_TF_IN_MESH) & ~GSIM_TF_ACTIVE);
    a.graft[sf.ir] = a.now;
    a.mtime[sf.ir] = 0;
}

__device__ __forceinline__ void stats_prune(const HbArgs& a, bool tracked, bool scored, double thr, double mcap,
                                            ScoreFlags& sf)
{
    if (!tracked || !scored || !sf.ok) return;
    uint8_t& fl = sf.get(a);
    if (fl & GSIM_TF_ACTIVE) {
        // pending delivery increments are part of the counter's value
        const double md = apply_incs(a.meshd[sf.ir], a.mcnt[sf.ir], mcap);
        if (md < thr) {
            const double deficit = thr - md;
            a.fail[sf.ir] = a.fail[sf.ir] + deficit * deficit;
        }
    }
    if (fl & GSIM_TF_IN_MESH) a.mtime[sf.ir] = 0;   // meshTime outside the mesh is 0
    fl &= (uint8_t)~GSIM_TF_IN_MESH;
}

// peerScore.score of one record (score.go:265-342), in the score pass's
// operation order: the live Score(p) emitGossip uses after this heartbeat's
// Graft/Prune changed the record (gossipsub.go:1734).
constexpr int kScoreChunk = 2;   // topics whose record fields are loaded together
// Diagnostic build (-DGSIM_DIAG_HB, counts only, results unchanged): [0]
// score_of_record calls, [1] Graft, [2] Prune, [3] backoff loads, summed over
// launches (gsim_diag_hb_counts)
#ifdef GSIM_DIAG_HB
__device__ unsigned long long g_hb_diag[4];
#endif

__device__ double score_of_record(const HbArgs& a_, uint32_t rv, uint32_t col)
{
    const HbArgs& a = hb_launder(a_);
    const uint8_t st = a.estate[rv];
    if (!(st & GSIM_ES_TRACKED)) return 0.0;
    // lazy meshTime (lazy_mtime): the graft times are loaded instead
    const int64_t* mts = a.mt_lazy ? a.graft : a.mtime;
    const uint64_t mj = smask_of(a.smask, col);      // the records sit in col's row
    const bool inv_zero = a.inv_live && !*a.inv_live;   // no record holds an invalid delivery
#ifdef GSIM_DIAG_HB
    atomicAdd(&g_hb_diag[0], 1ull);
#endif
    double score = 0.0;
    for (int32_t t0 = 0; t0 < a.T; t0 += kScoreChunk) {
        // the records sit at rv in each topic plane, away from the row: load a
        // chunk of topics before using any (one memory round trip per chunk)
        uint8_t fl[kScoreChunk], mc[kScoreChunk];
        double f[kScoreChunk], md[kScoreChunk], fa[kScoreChunk], iv[kScoreChunk];
        int64_t mt[kScoreChunk];
#pragma unroll
        for (int j = 0; j < kScoreChunk; ++j) {
            const int32_t t = t0 + j;
            const bool ok = t < a.T && (const_tp(a.tp) + t)->scored && slot_has(mj, t);
            const int64_t i = slot_idx(mj, t, a.E, rv);
            fl[j] = ok ? a.tflags[i] : 0;
            mc[j] = ok ? a.mcnt[i] : 0;
            f[j] = ok ? a.first[i] : 0.0;
            md[j] = ok ? a.meshd[i] : 0.0;
            fa[j] = ok ? a.fail[i] : 0.0;
            iv[j] = ok && !inv_zero ? a.invalid[i] : 0.0;
            mt[j] = ok ? mts[i] : 0;
        }
        for (int j = 0; j < kScoreChunk; ++j) {
            const int32_t t = t0 + j;
            if (t >= a.T) break;
            const ctp_t tp = const_tp(a.tp) + t;
            if (!tp->scored || !slot_has(mj, t)) continue;
            const double meshd = apply_incs(md[j], mc[j], tp->mesh_message_deliveries_cap);
            double ts = 0.0;
            if (fl[j] & GSIM_TF_IN_MESH) {                                // P1
                if (a.mt_lazy)
                    mt[j] = (st & GSIM_ES_CONNECTED) && mt[j] <= a.mt_R ? a.mt_R - mt[j]
                                                                       : a.mtime[slot_idx(mj, t, a.E, rv)];
                double p1 = 0.0;
                if (tp->time_in_mesh_quantum_ns != 0) p1 = (double)go_div(mt[j], tp->time_in_mesh_quantum_ns);
                if (p1 > tp->time_in_mesh_cap) p1 = tp->time_in_mesh_cap;
                ts += p1 * tp->time_in_mesh_weight;
            }
            ts += f[j] * tp->first_message_deliveries_weight;              // P2
            if (fl[j] & GSIM_TF_ACTIVE) {                                  // P3
                if (meshd < tp->mesh_message_deliveries_threshold) {
                    const double deficit = tp->mesh_message_deliveries_threshold - meshd;
                    const double p3 = deficit * deficit;
                    ts += p3 * tp->mesh_message_deliveries_weight;
                }
            }
            ts += fa[j] * tp->mesh_failure_penalty_weight;                 // P3b
            const double p4 = iv[j] * iv[j];                               // P4
            ts += p4 * tp->invalid_message_deliveries_weight;
            score += ts * tp->topic_weight;
        }
    }
    if (a.topic_cap > 0 && score > a.topic_cap) score = a.topic_cap;
    score += a.p5[col] * a.w5;                                         // P5
    score += a.p6[rv] * a.w6;                                          // P6
    const double bp = a.bp[rv];
    if (bp > a.bp_thr) {                                               // P7
        const double excess = bp - a.bp_thr;
        const double p7 = excess * excess;
        score += p7 * a.w7;
    }
    return score;
}

// emitGossip's target choice over the list L = candidates (key P_GOSSIP)
// followed, when fewer than Dlo, by fill instances (key P_GOSSIP_DUP) of
// the topic peers taken in P_GOSSIP_FILL order (gossipsub.go:1739-1762):
// target = max(Dlazy, int(GossipFactor * |L|)), all of L if that is not
// smaller, else the target smallest keys.  A lane is selected if any of its
// instances is.  Must be called by the whole wave.
template <int W = 64>
__device__ bool gossip_targets(const HbArgs& a, bool cand, bool tpeer, uint32_t obs, int32_t t, uint32_t col,
                               uint32_t pos, uint64_t gm = ~0ull, int grp = 0)
{
    const int c = __popcll(__ballot(cand) & gm);
    bool dup = false;
    if (c < a.Dlo) dup = select_smallest<W>(a, tpeer, a.Dlo - c, obs, t, P_GOSSIP_FILL, col, pos, gm, grp);
    const int n = c + __popcll(__ballot(dup) & gm);
    if (n == 0) return false;
    int target = a.dlazy;
    const int factor = (int)(a.gossip_factor * (double)n);
    if (factor > target) target = factor;
    if (target >= n) return cand || dup;
    // each lane holds up to two instances (candidate, fill duplicate)
    // no fill duplicates (the usual case): one instance per lane
    if (!(__ballot(dup) & gm)) return select_smallest<W>(a, cand, target, obs, t, P_GOSSIP, col, pos, gm, grp);
    uint32_t h1 = cand ? hb_key_hi(a, obs, t, P_GOSSIP, col, pos) : 0xFFFFFFFFu;
    uint32_t h2 = dup ? hb_key_hi(a, obs, t, P_GOSSIP_DUP, col, pos) : 0xFFFFFFFFu;
    uint64_t av1 = __ballot(cand) & gm, av2 = __ballot(dup) & gm;
    const int lane = threadIdx.x & 63;
    bool sel = false;
    for (int q = 0; q < target; ++q) {
        // a lane's next instance: its smaller key (instance 1 on a tie)
        const bool has1 = (av1 >> lane) & 1ull, has2 = (av2 >> lane) & 1ull;
        const bool use1 = has1 && (!has2 || h1 <= h2);
        const uint32_t mine = use1 ? h1 : (has2 ? h2 : 0xFFFFFFFFu);
        const uint32_t mn = group_min_u32<W>(mine, grp);
        const bool at_min = mine == mn && (has1 || has2);
        const int win = __ffsll((long long)(__ballot(at_min) & gm)) - 1;
        // which instance the winner used, from a ballot (no lane shuffle)
        if ((__ballot(at_min && use1) >> win) & 1ull) av1 &= ~(1ull << win); else av2 &= ~(1ull << win);
        if (lane == win) sel = true;
    }
    return sel;
}



// ---------------------------------------------------------------------------
// The lane group that holds one observer's row.  The heartbeat body
// (hb_observer) is written once against this interface:
//   WaveGroup<W>     W lanes of a wavefront (rows of at most 16 / 32 / 64
//                    connections; 4 / 2 / 1 observers per wavefront)
//   BlockGroup<B, V> a whole B-thread block holding V row positions per
//                    thread (hub rows of 65 .. B·V connections): counts and
//                    keyed minima are block reductions through LDS, a
//                    position's neighbours are read from LDS, not shuffles.
// Position q of a group is the row position (tie breaks, Philox keys); a
// thread holds positions pos(0) .. pos(V-1), and every per-position value
// crosses the interface as an array of V.

template <int W>
struct WaveGroup {
    static constexpr int V = 1;
    static constexpr int LP = 64 / W;     // topics per lane of the mcache-put cache
    int lane, grp, gl, base;
    uint64_t gm;
    int32_t lpv[LP];
    __device__ explicit WaveGroup(int lane_)
        : lane(lane_), grp(lane_ / W), gl(lane_ % W), base((lane_ / W) * W),
          gm(W == 64 ? ~0ull : (((1ull << W) - 1) << ((lane_ / W) * W)))
    {
    }
    __device__ int pos(int = 0) const { return gl; }
    __device__ int span() const { return W; }
    __device__ int count(const bool* p) const { return __popcll(__ballot(p[0]) & gm); }
    __device__ bool any(const bool* p) const { return (__ballot(p[0]) & gm) != 0; }
    __device__ void select(const HbArgs& a, const bool* cand, int count, uint32_t obs, int32_t t, uint32_t purpose,
                           const uint32_t* col, bool* out)
    {
        out[0] = select_smallest<W>(a, cand[0], count, obs, t, purpose, col[0], (uint32_t)gl, gm, grp);
    }
    __device__ void gossip(const HbArgs& a, const bool* cand, const bool* tpeer, uint32_t obs, int32_t t,
                           const uint32_t* col, bool* out)
    {
        out[0] = gossip_targets<W>(a, cand[0], tpeer[0], obs, t, col[0], (uint32_t)gl, gm, grp);
    }
    // a lane's value at position q of the group (every lane asks for the same q)
    template <typename T>
    struct View {
        T v;
        int base;
        __device__ T operator[](int q) const { return __shfl(v, base + q, 64); }
    };
    struct BoolView {
        uint64_t m;
        int base;
        __device__ bool operator[](int q) const { return (m >> (base + q)) & 1ull; }
    };
    template <int SLOT, typename T>
    __device__ View<T> view(const T* v) const { return View<T>{v[0], base}; }
    template <int SLOT>
    __device__ BoolView view_b(const bool* v) const { return BoolView{__ballot(v[0]), base}; }
    static constexpr bool kList = false;  // rank loops over every position (shuffles: the whole group)
    // the value at the lowest position where p holds (p must hold somewhere)
    __device__ double at_lowest(const bool* p, const double* v) const
    {
        return __shfl(v[0], (int)__ffsll((long long)(__ballot(p[0]) & gm)) - 1, 64);
    }
    // newest mcache put of topic t by observer obs (GetGossipIDs non-empty test):
    // group lane gl caches topics gl, gl + W, ... (T <= 64)
    // bit q = p at position q < 64 (W = 64: the wave's ballot)
    __device__ uint64_t topic_mask(bool p) const { return __ballot(p) & gm; }
    // bit q = p at the group's row position q (the delivery's mesh masks)
    static constexpr bool kRowMask = true;
    __device__ uint64_t row_mask(const bool* p) const { return (__ballot(p[0]) & gm) >> base; }
    __device__ void load_lastput(const HbArgs& a, int64_t obs, uint64_t subi, bool ovalid)
    {
#pragma unroll
        for (int k = 0; k < LP; ++k) {
            const int32_t t = gl + W * k;
            lpv[k] = (a.gossip && ovalid && t < a.T && ((subi >> t) & 1ull)) ? a.lastput[(int64_t)t * a.N + obs] : -1;
        }
    }
    __device__ int32_t lastput(const HbArgs&, int64_t, int32_t t) const
    {
        int32_t lpsel = lpv[0];
#pragma unroll
        for (int k = 1; k < LP; ++k)
            if (t >= W * k) lpsel = lpv[k];
        return __shfl(lpsel, base + (t & (W - 1)), 64);
    }
};

template <int B, int VV = 1>
struct BlockGroup {
    static constexpr int V = VV;
    static constexpr int NW = B / 64;
    static constexpr int P = B * V;       // positions
    struct Shared {
        unsigned long long red[2][NW];     // reductions (alternating: one barrier each)
        double d0[P];
        uint64_t u0[P], u1[P];
        int32_t i0[P];
        int32_t l0[P];                     // each(): positions where a predicate holds
        int ln;
        uint8_t b0[P], b1[P];
    };
    Shared* sh;
    int tid, lane, wid, phase;
    __device__ BlockGroup(Shared* s) : sh(s), tid((int)threadIdx.x), lane((int)threadIdx.x & 63),
                                       wid((int)threadIdx.x >> 6), phase(0) {}
    __device__ int pos(int v = 0) const { return v * B + tid; }
    __device__ int span() const { return P; }
    __device__ unsigned long long reduce(unsigned long long v, int op)   // 0 sum, 1 min, 2 max
    {
        for (int o = 32; o; o >>= 1) {
            const unsigned long long y = (unsigned long long)__shfl_xor((long long)v, o, 64);
            v = op == 0 ? v + y : op == 1 ? (y < v ? y : v) : (y > v ? y : v);
        }
        unsigned long long* r = sh->red[phase & 1];
        ++phase;
        if (lane == 0) r[wid] = v;
        __syncthreads();
        unsigned long long acc = r[0];
        for (int w = 1; w < NW; ++w) {
            const unsigned long long y = r[w];
            acc = op == 0 ? acc + y : op == 1 ? (y < acc ? y : acc) : (y > acc ? y : acc);
        }
        return acc;
    }
    __device__ int count(const bool* p)
    {
        unsigned long long c = 0;
#pragma unroll
        for (int v = 0; v < V; ++v) c += (unsigned long long)__popcll(__ballot(p[v]));
        return (int)reduce(c * (lane == 0), 0);
    }
    __device__ bool any(const bool* p) { return count(p) != 0; }
    __device__ uint64_t min_u64(uint64_t v) { return reduce(v, 1); }
    __device__ uint64_t max_u64(uint64_t v) { return reduce(v, 2); }
    // select_smallest (above) over the block: the count smallest (key, position)
    __device__ void select(const HbArgs& a, const bool* cand, int count, uint32_t obs, int32_t t, uint32_t purpose,
                           const uint32_t* col, bool* sel)
    {
        const int n = this->count(cand);
#pragma unroll
        for (int v = 0; v < V; ++v) sel[v] = false;
        if (n == 0) return;
        if (count <= 0 || n <= count) {
#pragma unroll
            for (int v = 0; v < V; ++v) sel[v] = cand[v];
            return;
        }
        const uint32_t tau = (uint32_t)((float)count / (float)n * 4294967040.0f);
        uint64_t key[V];
        bool rest[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const uint32_t hi = cand[v] ? hb_key_hi(a, obs, t, purpose, col[v], (uint32_t)pos(v)) : 0xFFFFFFFFu;
            key[v] = ((uint64_t)hi << 32) | (uint32_t)pos(v);
            sel[v] = cand[v] && hi < tau;
        }
        int c = this->count(sel);
        while (c > count) {                 // drop the largest (key, position) among the selected
            uint64_t mine = 0;
#pragma unroll
            for (int v = 0; v < V; ++v) if (sel[v] && key[v] > mine) mine = key[v];
            const uint64_t mx = max_u64(mine);
#pragma unroll
            for (int v = 0; v < V; ++v) if (sel[v] && key[v] == mx) sel[v] = false;
            --c;
        }
#pragma unroll
        for (int v = 0; v < V; ++v) rest[v] = cand[v] && !sel[v];
        while (c < count) {                 // add the smallest among the others
            uint64_t mine = ~0ull;
#pragma unroll
            for (int v = 0; v < V; ++v) if (rest[v] && key[v] < mine) mine = key[v];
            const uint64_t mn = min_u64(mine);
#pragma unroll
            for (int v = 0; v < V; ++v) if (rest[v] && key[v] == mn) { sel[v] = true; rest[v] = false; }
            ++c;
        }
    }
    // gossip_targets (above) over the block
    __device__ void gossip(const HbArgs& a, const bool* cand, const bool* tpeer, uint32_t obs, int32_t t,
                           const uint32_t* col, bool* sel)
    {
        const int c = count(cand);
        bool dup[V];
#pragma unroll
        for (int v = 0; v < V; ++v) { dup[v] = false; sel[v] = false; }
        if (c < a.Dlo) select(a, tpeer, a.Dlo - c, obs, t, P_GOSSIP_FILL, col, dup);
        const int n = c + count(dup);
        if (n == 0) return;
        int target = a.dlazy;
        const int factor = (int)(a.gossip_factor * (double)n);
        if (factor > target) target = factor;
        if (target >= n) {
#pragma unroll
            for (int v = 0; v < V; ++v) sel[v] = cand[v] || dup[v];
            return;
        }
        if (!any(dup)) { select(a, cand, target, obs, t, P_GOSSIP, col, sel); return; }
        uint32_t h1[V], h2[V];
        bool has1[V], has2[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            h1[v] = cand[v] ? hb_key_hi(a, obs, t, P_GOSSIP, col[v], (uint32_t)pos(v)) : 0xFFFFFFFFu;
            h2[v] = dup[v] ? hb_key_hi(a, obs, t, P_GOSSIP_DUP, col[v], (uint32_t)pos(v)) : 0xFFFFFFFFu;
            has1[v] = cand[v];
            has2[v] = dup[v];
        }
        for (int q = 0; q < target; ++q) {
            uint64_t k[V], mine = ~0ull;
            bool use1[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                use1[v] = has1[v] && (!has2[v] || h1[v] <= h2[v]);
                const uint32_t hv = use1[v] ? h1[v] : (has2[v] ? h2[v] : 0xFFFFFFFFu);
                k[v] = (has1[v] || has2[v]) ? (((uint64_t)hv << 32) | (uint32_t)pos(v)) : ~0ull;
                if (k[v] < mine) mine = k[v];
            }
            const uint64_t mn = min_u64(mine);
#pragma unroll
            for (int v = 0; v < V; ++v)
                if ((has1[v] || has2[v]) && k[v] == mn) {
                    if (use1[v]) has1[v] = false; else has2[v] = false;
                    sel[v] = true;
                }
        }
    }
    template <typename T>
    struct View {
        const T* p;
        __device__ T operator[](int q) const { return p[q]; }
    };
    template <int SLOT, typename T>
    __device__ View<T> view(const T* v)
    {
        T* buf;
        if constexpr (sizeof(T) == 8 && (T)0.5 != (T)0) buf = reinterpret_cast<T*>(sh->d0);     // double
        else if constexpr (sizeof(T) == 8) buf = reinterpret_cast<T*>(SLOT ? sh->u1 : sh->u0);
        else buf = reinterpret_cast<T*>(sh->i0);
        __syncthreads();                    // earlier readers of the buffer are done
#pragma unroll
        for (int x = 0; x < V; ++x) buf[pos(x)] = v[x];
        __syncthreads();
        return View<T>{buf};
    }
    template <int SLOT>
    __device__ View<uint8_t> view_b(const bool* v)
    {
        uint8_t* buf = SLOT ? sh->b1 : sh->b0;
        __syncthreads();
#pragma unroll
        for (int x = 0; x < V; ++x) buf[pos(x)] = v[x] ? 1 : 0;
        __syncthreads();
        return View<uint8_t>{buf};
    }
    // f(q) for the positions q where p holds, in no particular order: a hub's
    // rank loops count over its mesh, not its whole row (c5's hubs: rows of
    // thousands, meshes of tens)
    static constexpr bool kList = true;
    template <class F>
    __device__ void each(const bool* p, F f)
    {
        __syncthreads();                    // earlier readers of the list are done
        if (tid == 0) sh->ln = 0;
        __syncthreads();
#pragma unroll
        for (int x = 0; x < V; ++x)
            if (p[x]) sh->l0[atomicAdd(&sh->ln, 1)] = pos(x);
        __syncthreads();
        const int n = sh->ln;
        for (int j = 0; j < n; ++j) f(sh->l0[j]);
    }
    __device__ double at_lowest(const bool* p, const double* v)
    {
        uint64_t mine = ~0ull;
#pragma unroll
        for (int x = V - 1; x >= 0; --x) if (p[x]) mine = (uint64_t)pos(x);
        const uint64_t q = min_u64(mine);
        __syncthreads();
#pragma unroll
        for (int x = 0; x < V; ++x) if ((uint64_t)pos(x) == q) sh->d0[0] = v[x];
        __syncthreads();
        return sh->d0[0];
    }
    static constexpr bool kRowMask = false;    // hub rows: delivery walks the whole row
    __device__ uint64_t row_mask(const bool*) const { return 0; }
    __device__ uint64_t topic_mask(bool p)
    {
        const uint64_t m = __ballot(p);
        return reduce((wid == 0 && lane == 0) ? m : 0ull, 0);
    }
    __device__ void load_lastput(const HbArgs&, int64_t, uint64_t, bool) {}
    __device__ int32_t lastput(const HbArgs& a, int64_t obs, int32_t t) const
    {
        return a.lastput[(int64_t)t * a.N + obs];
    }
};

}  // namespace

// One observer's heartbeat (gossipsub.go:1345-1557) on its lane group:
// position q holds the observer's q-th connection; counts, selections and
// the neighbours' values go through the group (WaveGroup: ballots masked to
// the group, shuffles of the group's own lanes; BlockGroup: LDS).  Branches
// diverge only between whole groups.
template <class Grp>
__device__ __forceinline__ void hb_observer(const HbArgs& a_, Grp& g, int64_t obs, bool ovalid)
{
        const HbArgs& a = a_;
        constexpr int V = Grp::V;
        const uint32_t b = ovalid ? a.row_ptr[obs] : 0u;
        const int deg = ovalid ? (int)(a.row_ptr[obs + 1] - b) : 0;
        const uint32_t gobs = ovalid ? glob(a, (uint32_t)obs) : 0u;
        const uint64_t subi = ovalid ? a.sub[obs] : 0ull;
        // topic slots: router state is the observer's row (mi), its records of
        // the neighbours sit in their rows (mj, per position)
        const uint64_t mi = ovalid ? smask_of(a.smask, (uint32_t)obs) : 0ull;
        // per position v of this thread: row position g.pos(v)
        int gl[V];
        bool valid[V], tracked[V], conn[V], outb[V], dir[V], dirty[V];
        uint32_t e[V], col[V], rv[V], gcol[V];
        double S[V], S_live[V];
        uint64_t subj[V], mj[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            gl[v] = g.pos(v);
            valid[v] = gl[v] < deg;
            e[v] = b + (uint32_t)gl[v];
            col[v] = valid[v] ? a.col[e[v]] : 0u;
            rv[v] = valid[v] ? a.rev[e[v]] : 0u;           // this observer's record of col
            gcol[v] = valid[v] ? glob(a, col[v]) : 0u;
            const uint8_t est = valid[v] ? a.estate[rv[v]] : 0;
            tracked[v] = est & GSIM_ES_TRACKED;
            conn[v] = valid[v] && (a.rstate[e[v]] & GSIM_ES_CONNECTED);
            outb[v] = valid[v] && a.outbound[e[v]];
            dir[v] = valid[v] && a.direct[e[v]];          // direct peers are never grafted or gossiped to
            S[v] = valid[v] ? a.score[rv[v]] : 0.0;
            subj[v] = !valid[v] ? 0ull : a.sub_all ? ~0ull : a.sub[col[v]];
            mj[v] = valid[v] ? smask_of(a.smask, col[v]) : 0ull;
            // live score for emitGossip: the snapshot until this heartbeat's
            // Graft/Prune touches one of the position's records
            S_live[v] = S[v];
            dirty[v] = false;
            if (a.gossip && valid[v]) a.gstate[e[v]] = S[v] >= a.gossip_thr ? 1 : 0;
        }
        g.load_lastput(a, obs, subi, ovalid);
        uint64_t pxt = 0;                               // topics with a PRUNE carrying PX
        auto rescore = [&]() {                          // live scores of the dirty positions
            if (g.any(dirty)) {
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    if (dirty[v]) S_live[v] = score_of_record(a, rv[v], col[v]);
                    dirty[v] = false;
                }
            }
        };

        // clearBackoff every 15 ticks (gossipsub.go:1627-1646)
        if (a.tick % 15 == 0) {
#pragma unroll
            for (int v = 0; v < V; ++v) {
                if (!valid[v]) continue;
                for (int32_t t = 0; t < a.T; ++t) {
                    if (!slot_has(mi, t)) continue;
                    const int64_t i = slot_idx(mi, t, a.E, e[v]);
                    const int64_t bo = a.backoff[i];
                    if (bo != 0 && bo + kBackoffSlack < a.now) a.backoff[i] = 0;
                }
            }
        }

        for (int32_t t0 = 0; t0 < a.T; t0 += kFlagChunk) {
          // the flags of a chunk of topics are loaded together (one memory
          // round trip per chunk instead of one per topic); chunks without a
          // joined topic are skipped (a group-uniform test, like every
          // per-topic branch below)
          if (!((subi >> t0) & ((1ull << kFlagChunk) - 1))) continue;
          uint8_t flc[kFlagChunk][V];
#pragma unroll
          for (int j = 0; j < kFlagChunk; ++j) {
              const int32_t t = t0 + j;
#pragma unroll
              for (int v = 0; v < V; ++v)
                  flc[j][v] = (t < a.T && valid[v] && ((subi >> t) & 1ull)) ? a.mflags[slot_idx(mi, t, a.E, e[v])] : 0;
          }
          for (int j = 0; j < kFlagChunk; ++j) {
            const int32_t t = t0 + j;
            if (t >= a.T) break;
            if (!((subi >> t) & 1ull)) continue;           // not joined
            const HbArgs& a = hb_launder(a_);
            const ctp_t tp = const_tp(a.tp) + t;
            const bool scored = tp->scored != 0;
            const double thr = tp->mesh_message_deliveries_threshold;
            const double mcap = tp->mesh_message_deliveries_cap;
            int64_t i[V];
            ScoreFlags sf[V];
            uint8_t fl[V], fl0[V], ctl[V];
            // backoff is only consulted when a graft selection or a prune
            // happens, so it is loaded lazily (steady-state ticks read none)
            int64_t bo[V];
            bool have_bo[V], bo_dirty[V], tpeer[V], m[V], cand[V], sel[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                i[v] = slot_idx(mi, t, a.E, e[v]);
                sf[v].at(mj[v], t, a.E, rv[v]);
                fl[v] = flc[j][v];
                fl0[v] = fl[v];
                bo[v] = 0;
                have_bo[v] = bo_dirty[v] = false;
                tpeer[v] = valid[v] && conn[v] && ((subj[v] >> t) & 1ull);
                m[v] = valid[v] && (fl[v] & GSIM_TF_MESH);
                ctl[v] = 0;
            }
            auto need_bo = [&](int v) {
                if (!have_bo[v]) {
#ifdef GSIM_DIAG_HB
                    if (valid[v]) atomicAdd(&g_hb_diag[3], 1ull);
#endif
                    bo[v] = valid[v] ? a.backoff[i[v]] : 0;
                    have_bo[v] = true;
                }
            };
            auto prune = [&](int v) {
#ifdef GSIM_DIAG_HB
                atomicAdd(&g_hb_diag[2], 1ull);
#endif
                if (a.tr.on((uint32_t)obs)) a.tr.push(a.now, 0, (uint32_t)obs, col[v], t, GSIM_TRACE_PRUNE, 0);
                stats_prune(a, tracked[v], scored, thr, mcap, sf[v]);
                dirty[v] |= tracked[v] && scored;
                fl[v] &= (uint8_t)~GSIM_TF_MESH;
                m[v] = false;
                need_bo(v);
                const int64_t ex = a.now + a.prune_backoff;
                if (bo[v] < ex) { bo[v] = ex; bo_dirty[v] = true; }
                ctl[v] |= GSIM_CTL_PRUNE;
            };
            auto graft = [&](int v) {
#ifdef GSIM_DIAG_HB
                atomicAdd(&g_hb_diag[1], 1ull);
#endif
                if (a.tr.on((uint32_t)obs)) a.tr.push(a.now, 0, (uint32_t)obs, col[v], t, GSIM_TRACE_GRAFT, 0);
                stats_graft(a, tracked[v], scored, sf[v]);
                dirty[v] |= tracked[v] && scored;
                fl[v] |= GSIM_TF_MESH;
                m[v] = true;
                ctl[v] |= GSIM_CTL_GRAFT;
            };

            // drop all peers with negative score (1403-1410)
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (m[v] && S[v] < 0) prune(v);

            // too few peers: graft up to D (1412-1427)
            int l = g.count(m);
            if (l < a.Dlo) {
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    need_bo(v);
                    cand[v] = tpeer[v] && !m[v] && bo[v] == 0 && !dir[v] && S[v] >= 0;
                }
                g.select(a, cand, a.D - l, gobs, t, P_GRAFT_DLO, gcol, sel);
#pragma unroll
                for (int v = 0; v < V; ++v)
                    if (sel[v]) graft(v);
            }

            // too many peers: keep Dscore best + random, Dout outbound (1429-1490)
            l = g.count(m);
            if (l > a.Dhi) {
                uint64_t k1[V], k2[V];
                int rank1[V], below[V], p[V];
                bool tail[V];
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    k1[v] = m[v] ? hb_key(a, gobs, t, P_PRUNE_SHUF1, gcol[v], (uint32_t)gl[v]) : ~0ull;
                    rank1[v] = 0;
                }
                {
                    const auto vm = g.template view_b<0>(m);
                    const auto vs = g.template view<0>(S);
                    const auto vk = g.template view<0>(k1);
                    if constexpr (Grp::kList) {
                        g.each(m, [&](int q) {   // mesh positions: the only ones that count
                            const double sq = vs[q];
                            const uint64_t kq = vk[q];
                            const bool mq = vm[q];
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                if (mq && (sq > S[v] || (sq == S[v] && kq < k1[v]))) ++rank1[v];
                        });
                    } else {
                        for (int q = 0; q < g.span(); ++q) {
                            const double sq = vs[q];
                            const uint64_t kq = vk[q];
                            const bool mq = vm[q];
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                if (mq && (sq > S[v] || (sq == S[v] && kq < k1[v]))) ++rank1[v];
                        }
                    }
                }
                const int ds = a.Dscore < l ? a.Dscore : l;
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    tail[v] = m[v] && rank1[v] >= ds;
                    k2[v] = tail[v] ? hb_key(a, gobs, t, P_PRUNE_SHUF2, gcol[v], (uint32_t)gl[v]) : ~0ull;
                    below[v] = 0;
                }
                // every lane takes part in the shuffles (a shuffle inside a
                // divergent branch would read inactive lanes)
                {
                    const auto vk2 = g.template view<1>(k2);
                    if constexpr (Grp::kList) {
                        g.each(m, [&](int q) {   // mesh positions: the only ones that count
                            const uint64_t kq = vk2[q];
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                if (kq < k2[v]) ++below[v];   // non-tail positions hold ~0 and never count
                        });
                    } else {
                        for (int q = 0; q < g.span(); ++q) {
                            const uint64_t kq = vk2[q];
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                if (kq < k2[v]) ++below[v];   // non-tail positions hold ~0 and never count
                        }
                    }
                }
                // Keep plst[:D] after Go's Dout rotation (1457-1485), computed
                // data-parallel from each position's place p in plst:
                //  pass 1 moves every outbound peer at positions 1..D-1 to the
                //  front, leaving the other first-D peers ("rest") behind them
                //  in order; pass 2 rotates the first j outbound peers beyond D
                //  to the front, pushing the last j "rest" peers out of plst[:D].
                bool inD[V], keep[V], obc[V];
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    p[v] = tail[v] ? ds + below[v] : rank1[v];
                    inD[v] = m[v] && p[v] < a.D;
                    keep[v] = inD[v];
                    obc[v] = inD[v] && outb[v];
                }
                const int obD = g.count(obc);
                if (obD < a.Dout) {
                    bool rest[V], cb[V];
                    int rb[V], rr[V];
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        rest[v] = inD[v] && !(outb[v] && p[v] >= 1);
                        cb[v] = m[v] && p[v] >= a.D && outb[v];
                        rb[v] = rr[v] = 0;
                    }
                    const int nb = g.count(cb);
                    {
                        const auto vrest = g.template view_b<0>(rest);
                        const auto vcb = g.template view_b<1>(cb);
                        const auto vp = g.template view<0>(p);
                        if constexpr (Grp::kList) {
                            g.each(m, [&](int q) {   // mesh positions: the only ones that count
                                const int pq = vp[q];
                                const bool cq = vcb[q], rq = vrest[q];
#pragma unroll
                                for (int v = 0; v < V; ++v) {
                                    if (cq && pq < p[v]) ++rb[v];
                                    if (rq && pq > p[v]) ++rr[v];
                                }
                            });
                        } else {
                            for (int q = 0; q < g.span(); ++q) {
                                const int pq = vp[q];
                                const bool cq = vcb[q], rq = vrest[q];
#pragma unroll
                                for (int v = 0; v < V; ++v) {
                                    if (cq && pq < p[v]) ++rb[v];
                                    if (rq && pq > p[v]) ++rr[v];
                                }
                            }
                        }
                    }
                    const int jj = a.Dout - obD < nb ? a.Dout - obD : nb;
#pragma unroll
                    for (int v = 0; v < V; ++v) keep[v] = (inD[v] && !(rest[v] && rr[v] < jj)) || (cb[v] && rb[v] < jj);
                }
#pragma unroll
                for (int v = 0; v < V; ++v)
                    if (m[v] && !keep[v]) {
                        prune(v);
                        if (a.do_px) ctl[v] |= GSIM_CTL_PX;     // makePrune(p, topic, doPX && !noPX[p]) (1690)
                    }
            }

            // enough outbound peers? (1492-1518)
            l = g.count(m);
            if (l >= a.Dlo) {
                bool mo[V];
#pragma unroll
                for (int v = 0; v < V; ++v) mo[v] = m[v] && outb[v];
                const int ob = g.count(mo);
                if (ob < a.Dout) {
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        need_bo(v);
                        cand[v] = tpeer[v] && !m[v] && bo[v] == 0 && !dir[v] && outb[v] && S[v] >= 0;
                    }
                    g.select(a, cand, a.Dout - ob, gobs, t, P_GRAFT_DOUT, gcol, sel);
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (sel[v]) graft(v);
                }
            }

            // opportunistic grafting (1520-1552)
            l = g.count(m);
            if (a.opp_ticks && a.tick % a.opp_ticks == 0 && l > 1) {
                int rank[V];
#pragma unroll
                for (int v = 0; v < V; ++v) rank[v] = 0;
                {
                    const auto vm = g.template view_b<0>(m);
                    const auto vs = g.template view<0>(S);
                    if constexpr (Grp::kList) {
                        g.each(m, [&](int q) {   // mesh positions: the only ones that count
                            const double sq = vs[q];
                            const bool mq = vm[q];
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                if (mq && (sq < S[v] || (sq == S[v] && q < gl[v]))) ++rank[v];
                        });
                    } else {
                        for (int q = 0; q < g.span(); ++q) {
                            const double sq = vs[q];
                            const bool mq = vm[q];
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                if (mq && (sq < S[v] || (sq == S[v] && q < gl[v]))) ++rank[v];
                        }
                    }
                }
                bool atm[V];
#pragma unroll
                for (int v = 0; v < V; ++v) atm[v] = m[v] && rank[v] == l / 2;
                const double median = g.at_lowest(atm, S);
                if (median < a.opp_threshold) {
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        need_bo(v);
                        cand[v] = tpeer[v] && !m[v] && bo[v] == 0 && !dir[v] && S[v] > median;
                    }
                    g.select(a, cand, a.opp_peers, gobs, t, P_GRAFT_OPP, gcol, sel);
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (sel[v]) graft(v);
                }
            }

#pragma unroll
            for (int v = 0; v < V; ++v) {
                if (!valid[v]) continue;
                if (fl[v] != fl0[v]) a.mflags[i[v]] = fl[v];
                sf[v].store(a);
                if (bo_dirty[v]) a.backoff[i[v]] = bo[v];
            }
          {
            const HbArgs& a = hb_launder(a_);   // (the mesh maintenance's pointers are dead here)
            // the delivery's mesh mask of this row and topic (mesh or direct
            // edges to this shard's peers)
            if constexpr (Grp::kRowMask) {
                if (a.mmask) {
                    bool mm[V];
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        mm[v] = valid[v] && (m[v] || dir[v]) && col[v] >= a.mlo && col[v] < a.mhi;
                    const uint64_t mk = g.row_mask(mm);
                    if (gl[0] == 0 && ovalid) a.mmask[(int64_t)t * a.N + obs] = mk;
                }
            }

            // emitGossip(topic, mesh) (gossipsub.go:1554-1556, 1711-1775):
            // only if GetGossipIDs(topic) is non-empty, i.e. this peer put a
            // message of the topic in the last HistoryGossip ticks.  The
            // choice is stored in the sender's row (enqueueGossip); every
            // joined topic's plane is rewritten each heartbeat.
            if (a.gossip) {
                bool gs[V];
#pragma unroll
                for (int v = 0; v < V; ++v) gs[v] = false;
                const int32_t lpt = g.lastput(a, obs, t);
                if (lpt >= 0 && lpt >= (int64_t)a.tick - a.hist_gossip) {   // -1: no put yet
                    rescore();
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        cand[v] = tpeer[v] && !m[v] && !dir[v] && S_live[v] >= a.gossip_thr;
                    g.gossip(a, cand, tpeer, gobs, t, gcol, gs);
                }
#pragma unroll
                for (int v = 0; v < V; ++v)
                    if (valid[v]) a.gsel[i[v]] = gs[v] ? 1 : 0;
            }
            bool pxc[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                if (valid[v] && ctl[v] && slot_has(mj[v], t)) {
                    const int64_t r = slot_idx(mj[v], t, a.E, rv[v]);   // the receiver's row
                    a.ctl_out[r] = (uint8_t)(a.ctl_out[r] | ctl[v]);
                    atomicOr(reinterpret_cast<unsigned long long*>(a.cany_out + col[v]), 1ull << t);
                }
                pxc[v] = (ctl[v] & GSIM_CTL_PX) != 0;
            }
            if (a.do_px && g.any(pxc)) pxt |= 1ull << t;
          }
          }
        }
        // sendGraftPrune follows every topic: k_px_emit picks the PX peers
        if (a.do_px && pxt) {
            // the live scores makePrune's PX filter reads (k_px_emit): positions
            // this heartbeat's Graft/Prune touched since their last re-score
            rescore();
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (valid[v]) a.pxs[e[v]] = S_live[v];
            if (gl[0] == 0 && ovalid) a.pxo[obs] = pxt;
        }
}

// W-lane groups: W = 64 one observer per wavefront, W = 32 two, W = 16 four
// (rows of at most W connections; every VALU instruction serves G observers).
// rows: the observers of one row-length class (a list), or nullptr for the
// nrows observers from obs_base on.
template <int W>
// waves per SIMD the register budget is fitted to: 5 for W = 32 / 64 (C3's
// k_heartbeat<32>: 96 VGPRs with 10 spilled, 7.91 -> 6.81 ms per tick against 4
// waves at 106, 7.13 at 6; gpurun_out/r04pab, r04q), 4 for W = 16 (c5's
// heartbeat 116.8 -> 114.1 ms per tick against 3, r04qc5)
#ifndef GSIM_HB_WPE
#define GSIM_HB_WPE 5
#endif
#ifndef GSIM_HB_WPE16
#define GSIM_HB_WPE16 4
#endif
#ifndef GSIM_CHURN_MCNT
#define GSIM_CHURN_MCNT 1  // churn applies the pending meshd increments of the records it touches
#endif
#ifndef GSIM_HB_W8
#define GSIM_HB_W8 1       // rows of <= 8 connections in 8-lane groups (0: in the 16-lane class)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W <= 16 ? GSIM_HB_WPE16 : GSIM_HB_WPE)))
void k_heartbeat(HbArgs a, const uint32_t* rows, int64_t nrows, int64_t obs_base)
{
    constexpr int G = 64 / W;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    WaveGroup<W> g(lane);
    for (int64_t o0 = ((int64_t)blockIdx.x * 4 + wid) * G; o0 < nrows; o0 += (int64_t)gridDim.x * 4 * G) {
        const bool ovalid = o0 + g.grp < nrows;
        const int64_t obs = !ovalid ? 0 : rows ? (int64_t)rows[o0 + g.grp] : obs_base + o0 + g.grp;
        hb_observer(a, g, obs, ovalid);
    }
}

// Hub observers (rows of 65 .. B connections): one block per observer.
template <int B, int V>
__global__ __launch_bounds__(B) void k_heartbeat_hub(HbArgs a, const uint32_t* rows, int64_t nrows)
{
    __shared__ typename BlockGroup<B, V>::Shared sh;
    BlockGroup<B, V> g(&sh);
    for (int64_t o = blockIdx.x; o < nrows; o += gridDim.x) hb_observer(a, g, (int64_t)rows[o], true);
}

// ... rows of 4097..8192 connections: the same code over a group whose state
// is in global scratch (one slice per block; every view and reduction is a
// plain pointer access, ordered by the block's barriers)
template <int B, int V>
__global__ __launch_bounds__(B) void k_heartbeat_hub_g(HbArgs a, const uint32_t* rows, int64_t nrows, void* scratch)
{
    using S = typename BlockGroup<B, V>::Shared;
    BlockGroup<B, V> g(reinterpret_cast<S*>(scratch) + blockIdx.x);
    for (int64_t o = blockIdx.x; o < nrows; o += gridDim.x) hb_observer(a, g, (int64_t)rows[o], true);
}

// Fanout expiry and maintenance (gossipsub.go:1558-1596), run after
// k_heartbeat (the reference handles fanouts after every joined topic): drop
// the fanouts not published to for FanoutTTL; for each remaining fanout topic
// (ascending) drop peers that left the topic or score below
// publishThreshold, top up to D, and emitGossip excluding the fanout peers
// with the live score after this heartbeat's Graft/Prune.  One wave per
// observer; observers without fanout state leave after two loads.
template <class Grp>
__device__ __forceinline__ void fanout_observer(const HbArgs& a, Grp& g, int64_t obs)
{
        constexpr int V = Grp::V;
        const int gl0 = g.pos(0);
        const int64_t lpub = gl0 < a.T ? a.lastpub[obs * a.T + gl0] : 0;   // position 0 < 64 covers the topics
        const uint64_t expired = g.topic_mask(lpub != 0 && lpub + a.fanout_ttl < a.now);
        const uint64_t fant0 = a.fan_topics[obs];
        if (!expired && !fant0) return;                         // group-uniform
        const uint32_t b = a.row_ptr[obs];
        const int deg = (int)(a.row_ptr[obs + 1] - b);
        bool valid[V];
        uint32_t e[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            valid[v] = g.pos(v) < deg;
            e[v] = b + (uint32_t)g.pos(v);
        }
        if (gl0 < 64 && ((expired >> gl0) & 1ull)) a.lastpub[obs * a.T + gl0] = 0;
        const uint64_t mi = smask_of(a.smask, (uint32_t)obs);   // fanout topics hold slots (gsim_publish)
        for (uint64_t q = expired & fant0 & mi; q; q &= q - 1) {
#pragma unroll
            for (int v = 0; v < V; ++v) {
                if (!valid[v]) continue;
                const int64_t i = slot_idx(mi, __ffsll((long long)q) - 1, a.E, e[v]);
                const uint8_t fl = a.mflags[i];
                if (fl & GSIM_TF_FANOUT) a.mflags[i] = (uint8_t)(fl & ~GSIM_TF_FANOUT);
                if (a.gossip) a.gsel[i] = 0;                    // no more gossip for it
            }
        }
        const uint64_t fant = fant0 & ~expired;
        if (gl0 == 0 && fant != fant0) a.fan_topics[obs] = fant;
        if (!fant) return;
        const uint32_t gobs = glob(a, (uint32_t)obs);
        uint32_t col[V], rv[V], gcol[V];
        bool conn[V], dir[V];
        double S[V], S_live[V];
        uint64_t subj[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            col[v] = valid[v] ? a.col[e[v]] : 0u;
            rv[v] = valid[v] ? a.rev[e[v]] : 0u;
            gcol[v] = valid[v] ? glob(a, col[v]) : 0u;
            conn[v] = valid[v] && (a.rstate[e[v]] & GSIM_ES_CONNECTED);
            dir[v] = valid[v] && a.direct[e[v]];
            S[v] = valid[v] ? a.score[rv[v]] : 0.0;
            subj[v] = !valid[v] ? 0ull : a.sub_all ? ~0ull : a.sub[col[v]];
            S_live[v] = 0.0;
        }
        bool have_live = false;
        for (uint64_t q = fant & mi; q; q &= q - 1) {
            const int32_t t = __ffsll((long long)q) - 1;
            int64_t i[V];
            uint8_t fl[V];
            bool tpeer[V], inf[V], cand[V], sel[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                i[v] = slot_idx(mi, t, a.E, e[v]);
                fl[v] = valid[v] ? a.mflags[i[v]] : 0;
                tpeer[v] = conn[v] && ((subj[v] >> t) & 1ull);
                inf[v] = (fl[v] & GSIM_TF_FANOUT) && tpeer[v] && S[v] >= a.pub_thr;
            }
            const int have = g.count(inf);
            if (have < a.D) {
#pragma unroll
                for (int v = 0; v < V; ++v) cand[v] = tpeer[v] && !inf[v] && !dir[v] && S[v] >= a.pub_thr;
                g.select(a, cand, a.D - have, gobs, t, P_FANOUT, gcol, sel);
#pragma unroll
                for (int v = 0; v < V; ++v) if (sel[v]) inf[v] = true;
            }
#pragma unroll
            for (int v = 0; v < V; ++v) {
                const uint8_t nf = inf[v] ? (uint8_t)(fl[v] | GSIM_TF_FANOUT) : (uint8_t)(fl[v] & ~GSIM_TF_FANOUT);
                if (valid[v] && nf != fl[v]) a.mflags[i[v]] = nf;
            }
            if (!a.gossip) continue;
            bool gs[V];
#pragma unroll
            for (int v = 0; v < V; ++v) gs[v] = false;
            const int32_t lpt = a.lastput[(int64_t)t * a.N + obs];
            if (lpt >= 0 && lpt >= (int64_t)a.tick - a.hist_gossip) {
                if (!have_live) {                               // live Score(p), gossipsub.go:1734
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        if (valid[v]) S_live[v] = score_of_record(a, rv[v], col[v]);
                    have_live = true;
                }
#pragma unroll
                for (int v = 0; v < V; ++v) cand[v] = tpeer[v] && !inf[v] && !dir[v] && S_live[v] >= a.gossip_thr;
                g.gossip(a, cand, tpeer, gobs, t, gcol, gs);
            }
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (valid[v]) a.gsel[i[v]] = gs[v] ? 1 : 0;
        }
}

// Fanout expiry and maintenance, one wave per observer of at most 64
// connections; observers without fanout state leave after two loads.
__global__ __launch_bounds__(256) void k_fanout_heartbeat(HbArgs a_)
{
    const HbArgs& a = a_;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    WaveGroup<64> g(lane);
    for (int64_t obs = a.olo + (int64_t)blockIdx.x * 4 + wid; obs < a.ohi; obs += (int64_t)gridDim.x * 4) {
        if (a.row_ptr[obs + 1] - a.row_ptr[obs] > 64u) continue;    // a hub: k_fanout_heartbeat_hub
        fanout_observer(hb_launder(a_), g, obs);   // (re-read per observer: SGPR pressure)
    }
}

// ... of the hub observers (rows of 65 .. B connections), one block each
template <int B, int V>
__global__ __launch_bounds__(B) void k_fanout_heartbeat_hub(HbArgs a, const uint32_t* rows, int64_t nrows)
{
    __shared__ typename BlockGroup<B, V>::Shared sh;
    BlockGroup<B, V> g(&sh);
    for (int64_t o = blockIdx.x; o < nrows; o += gridDim.x) fanout_observer(a, g, (int64_t)rows[o]);
}

template <int B, int V>
__global__ __launch_bounds__(B) void k_fanout_heartbeat_hub_g(HbArgs a, const uint32_t* rows, int64_t nrows, void* scratch)
{
    using S = typename BlockGroup<B, V>::Shared;
    BlockGroup<B, V> g(reinterpret_cast<S*>(scratch) + blockIdx.x);
    for (int64_t o = blockIdx.x; o < nrows; o += gridDim.x) fanout_observer(a, g, (int64_t)rows[o]);
}

// HandleRPC control processing for every receiver: handleGraft
// (gossipsub.go:741-837) and handlePrune (839-871), senders in row order.
// The control records of one (receiver, topic) are usually few, so they are
// walked with a wave-uniform loop over the set bits of a ballot; the mesh size
// is carried in a scalar.
__global__ __launch_bounds__(256) void k_handle_control(HbArgs a_)
{
    const HbArgs& a = a_;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int64_t rcv = a.olo + (int64_t)blockIdx.x * 4 + wid; rcv < a.ohi; rcv += (int64_t)gridDim.x * 4) {
        // topics whose inbox planes may hold entries for this receiver: the
        // others are not read (most receivers get no GRAFT/PRUNE in a round)
        const uint64_t any = a.cany_in[rcv];
        if (!any) continue;
        if (lane == 0) a.cany_in[rcv] = 0;
        const uint32_t b = a.row_ptr[rcv];
        const int deg = (int)(a.row_ptr[rcv + 1] - b);
        const int nch = (deg + 63) >> 6;                    // rows longer than 64: 64-edge chunks in order
        const uint64_t subr = a.sub[rcv];
        const uint64_t mr = smask_of(a.smask, (uint32_t)rcv);   // the inbox and router state: rcv's row
        uint64_t pxo = 0;          // topics with a PRUNE reply carrying PX (mesh full, gossipsub.go:812-818)
        bool nopx_set = false;     // this lane marked a sender whose RPC turned PX off
        for (int32_t t0 = 0; t0 < a.T; t0 += kFlagChunk) {
          if (!((any >> t0) & ((1ull << kFlagChunk) - 1))) continue;
          for (int j = 0; j < kFlagChunk; ++j) {
            const int32_t t = t0 + j;
            if (t >= a.T) break;
            if (!((any >> t) & 1ull) || !slot_has(mr, t)) continue;
            const HbArgs& a = hb_launder(a_);   // (re-read per topic: SGPR pressure)
            const bool joined = (subr >> t) & 1ull;
            const ctp_t tp = const_tp(a.tp) + t;
            const bool scored = tp->scored != 0;
            const double thr = tp->mesh_message_deliveries_threshold;
            const double mcap = tp->mesh_message_deliveries_cap;
            // the mesh size before this round's records (the whole row)
            int mesh = 0;
            if (joined)
                for (int ch = 0; ch < nch; ++ch) {
                    const bool v = ch * 64 + lane < deg;
                    mesh += __popcll(ballot(v && (a.mflags[slot_idx(mr, t, a.E, b + ch * 64 + lane)] & GSIM_TF_MESH)));
                }
            for (int ch = 0; ch < nch; ++ch) {
              const bool valid = ch * 64 + lane < deg;
              const uint32_t e = b + (uint32_t)(ch * 64 + lane);
              const int64_t i = slot_idx(mr, t, a.E, e);
              const uint8_t c = valid ? a.ctl_in[i] : 0;
              uint64_t pending = ballot(c != 0);
              if (!pending) continue;
              if (c) a.ctl_in[i] = 0;
              if (!joined) {                                  // unknown topic: ignored, no PX (753-759)
                  if (a.do_px && (c & GSIM_CTL_GRAFT)) { a.nopx[e] = 1; nopx_set = true; }
                  continue;
              }
              uint8_t fl = valid ? a.mflags[i] : 0;
              while (pending) {
                const int q = __ffsll((long long)pending) - 1;
                pending &= pending - 1;
                int delta = 0, pxr = 0;
                if (lane == q) {
                    const uint8_t fl_in = fl;
                    const uint32_t rv = a.rev[e];                // receiver's record of the sender
                    const uint8_t est = a.estate[rv];
                    const bool tracked = est & GSIM_ES_TRACKED;
                    const uint64_t mj = smask_of(a.smask, a.col[e]);   // the sender's row
                    ScoreFlags sf;
                    sf.at(mj, t, a.E, rv);
                    int64_t bo = a.backoff[i];
                    const int64_t bo0 = bo;
                    uint8_t reply = 0;
                    if ((c & GSIM_CTL_GRAFT) && !(fl & GSIM_TF_MESH)) {
                        bool off = true;                     // doPX = false for the RPC
                        if (a.direct[e]) {
                            // no GRAFT to/from direct peers: answered with PRUNE (gossipsub.go:768-776)
                            reply = GSIM_CTL_PRUNE;
                        } else if (bo != 0 && a.now < bo) {
                            // GRAFT while backing off: P7 penalty (+1 more under the flood cutoff)
                            if (tracked) {
                                double x = a.bp[rv] + 1.0;
                                if (a.now < bo + (a.graft_flood - a.prune_backoff)) x = x + 1.0;
                                a.bp[rv] = x;
                            }
                            const int64_t ex = a.now + a.prune_backoff;
                            if (bo < ex) bo = ex;
                            reply = GSIM_CTL_PRUNE;
                        } else if (a.score[rv] < 0) {
                            reply = GSIM_CTL_PRUNE;
                            const int64_t ex = a.now + a.prune_backoff;
                            if (bo < ex) bo = ex;
                        } else if (mesh >= a.Dhi && !a.outbound[e]) {
                            reply = (uint8_t)(GSIM_CTL_PRUNE | (a.do_px ? GSIM_CTL_PX : 0));
                            pxr = a.do_px;
                            off = false;
                            const int64_t ex = a.now + a.prune_backoff;
                            if (bo < ex) bo = ex;
                        } else {
                            if (a.tr.on((uint32_t)rcv)) a.tr.push(a.now, 0, (uint32_t)rcv, a.col[e], t, GSIM_TRACE_GRAFT, 0);
                            stats_graft(a, tracked, scored, sf);
                            fl |= GSIM_TF_MESH;
                            delta += 1;
                            off = false;
                        }
                        if (a.do_px && off) { a.nopx[e] = 1; nopx_set = true; }
                    }
                    if (c & GSIM_CTL_PRUNE) {
                        // handlePrune: tracer.Prune whether or not the sender was in the mesh (gossipsub.go:849-851)
                        if (a.tr.on((uint32_t)rcv)) a.tr.push(a.now, 0, (uint32_t)rcv, a.col[e], t, GSIM_TRACE_PRUNE, 0);
                        if (fl & GSIM_TF_MESH) delta -= 1;
                        stats_prune(a, tracked, scored, thr, mcap, sf);
                        fl &= (uint8_t)~GSIM_TF_MESH;
                        // the PRUNE's Backoff: PruneBackoff/1s, or UnsubscribeBackoff/1s for Leave's
                        const int64_t secs = ((c & GSIM_CTL_UNSUB) ? a.unsub_backoff : a.prune_backoff) / kSecond;
                        const int64_t ex = a.now + (secs > 0 ? secs * kSecond : a.prune_backoff);
                        if (bo < ex) bo = ex;
                    }
                    a.mflags[i] = fl;
                    if (a.rdel && ((fl ^ fl_in) & GSIM_TF_MESH) && a.xq[e] != 0xFFFFFFFFu) {
                        // a cross edge: its copy in the other shard's ghost row changes
                        const uint32_t cj = a.col[e];
                        uint32_t dsh = 0;
                        while ((int32_t)dsh + 1 < a.sr.K && (int64_t)cj >= a.sr.lo[dsh + 1]) ++dsh;
                        const uint32_t pos = atomicAdd(a.rdel_n, 1u);
                        if ((int64_t)pos < a.rdel_cap)
                            a.rdel[pos] = (uint64_t)a.sr.self | ((uint64_t)dsh << 6) | ((uint64_t)t << 12) |
                                          ((uint64_t)(fl & (GSIM_TF_MESH | GSIM_TF_FANOUT)) << 20) |
                                          ((uint64_t)a.xq[e] << 32);
                    }
                    sf.store(a);
                    if (bo != bo0) a.backoff[i] = bo;
                    if (reply && slot_has(mj, t)) {
                        const int64_t r = slot_idx(mj, t, a.E, rv);
                        a.ctl_out[r] = (uint8_t)(a.ctl_out[r] | reply);
                        atomicOr(reinterpret_cast<unsigned long long*>(a.cany_out + a.col[e]), 1ull << t);
                    }
                }
                mesh += __shfl(delta, q, 64);
                if (__shfl(pxr, q, 64)) pxo |= 1ull << t;
              }
              if (nch == 1 && a.mmask) {                      // the delivery's mesh mask of the row
                  const uint32_t cj = valid ? a.col[e] : 0u;
                  const uint64_t mk = ballot(valid && ((fl & GSIM_TF_MESH) || a.direct[e]) && cj >= a.mlo && cj < a.mhi);
                  if (lane == 0) a.mmask[(int64_t)t * a.N + rcv] = mk;
              }
            }
          }
        }
        if (a.do_px && (pxo || ballot(nopx_set))) {
            // a sender whose RPC turned PX off gets its PRUNE replies without PX
            // (doPX is per handleGraft call, gossipsub.go:744-834); the marks are reset
            for (int ch = 0; ch < nch; ++ch) {
                const bool valid = ch * 64 + lane < deg;
                const uint32_t e = b + (uint32_t)(ch * 64 + lane);
                if (!valid || !a.nopx[e]) continue;
                a.nopx[e] = 0;
                const uint32_t re = a.rev[e];
                const uint64_t mj = smask_of(a.smask, a.col[e]);
                for (uint64_t q = pxo & mj; q; q &= q - 1) {
                    const int64_t r = slot_idx(mj, __ffsll((long long)q) - 1, a.E, re);
                    a.ctl_out[r] = (uint8_t)(a.ctl_out[r] & ~GSIM_CTL_PX);
                }
            }
            if (lane == 0 && pxo) a.pxo[rcv] = pxo;
        }
    }
}

// makePrune's peer exchange and the pruned peer's handlePrune / pxConnect
// (gossipsub.go:1866-1906, 860-869, 893-939) for the PRUNEs an observer just
// sent with PX (GSIM_CTL_PX in ctl_out; pxo[obs] lists their topics): the
// PX list is getPeers(topic, PrunePeers, xp != p && Score(xp) >= 0), the
// PrunePeers smallest keys (px_key: the topic's draw per candidate, px_base,
// mixed with the pruned peer's row position: every PRUNE its own shuffle).  live: Score is the observer's
// live score (the heartbeat's sendGraftPrune, after every topic); else the
// snapshot (the control round's GRAFT replies).  The pruned
// peer ignores PX from a peer it scores below acceptPXThreshold; every listed
// peer with a known address (an edge of its row) is a connection attempt
// (pxm), resolved between ticks by gsim_px_connect.  One wave per observer;
// rows of at most 1024 connections (keys and scores staged in LDS).
constexpr int kPxRow = 1024;
constexpr int kPxList = 64;     // keys a PRUNE lists below its bound (one per lane)

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v)
{
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = (uint64_t)__shfl_xor((long long)v, o, 64);
        v = y > v ? y : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v)
{
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = (uint64_t)__shfl_xor((long long)v, o, 64);
        v = y < v ? y : v;
    }
    return v;
}

// LDS written by some lanes of a wave, read by others
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ROW: the longest row staged (WV waves per block, ROW scores and keys each):
// <kPxRow, 4> walks the owned observers with rows of at most kPxRow,
// <4 kPxRow, 1> the hub list `rows` (rows of kPxRow+1 .. 4 kPxRow).
template <int ROW, int WV, bool SPLIT = false>
__global__ __launch_bounds__(64 * WV) void k_px_emit(HbArgs a_, int live, uint32_t key_tick, uint32_t purpose,
                                                     const uint32_t* rows, int64_t nrows)
{
    const HbArgs& a = a_;
    // SPLIT (hub rows): the block's waves share one observer (its scores, each
    // topic's candidates and draws) and take its PRUNEs in turn
    __shared__ double s_sc[SPLIT ? 1 : WV][ROW];
    __shared__ uint64_t s_cb[SPLIT ? 1 : WV][ROW / 64];          // the topic's candidates (makePrune's filter)
    __shared__ uint32_t s_pb[SPLIT ? 1 : WV][ROW];               // ... and their draws (px_base)
    __shared__ uint64_t s_lst[WV][kPxList];                      // a PRUNE's smallest keys
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double* sc = s_sc[SPLIT ? 0 : wid];
    uint64_t* cb = s_cb[SPLIT ? 0 : wid];
    uint32_t* pb = s_pb[SPLIT ? 0 : wid];
    uint64_t* lst = s_lst[wid];
    const int64_t nobs = rows ? nrows : a.ohi - a.olo;
    constexpr int OPB = SPLIT ? 1 : WV;                          // observers per block
    const int slot = SPLIT ? 0 : wid;
    for (int64_t x = (int64_t)blockIdx.x * OPB + slot; x < nobs; x += (int64_t)gridDim.x * OPB) {
        const int64_t obs = rows ? (int64_t)rows[x] : a.olo + x;
        const uint32_t b = a.row_ptr[obs];
        const int deg = (int)(a.row_ptr[obs + 1] - b);
        if (deg > ROW) continue;                                 // a longer hub: the hub instances
        const uint64_t mask = a.pxo[obs];
        if (!mask) continue;
        const uint32_t gobs = glob(a, (uint32_t)obs);
        if constexpr (SPLIT) {
            for (int q = threadIdx.x; q < deg; q += 64 * WV) sc[q] = live ? a.pxs[b + (uint32_t)q] : a.score[a.rev[b + (uint32_t)q]];
            __syncthreads();                                     // (every wave has read the mask too)
            if (threadIdx.x == 0) a.pxo[obs] = 0;
        } else {
            if (lane == 0) a.pxo[obs] = 0;
            for (int q = lane; q < deg; q += 64) {
                const uint32_t e = b + (uint32_t)q, rv = a.rev[e];
                sc[q] = live ? a.pxs[e] : a.score[rv];
            }
            wave_lds_sync();
        }
        int turn = 0;                                            // SPLIT: the PRUNEs dealt to the waves in turn
        for (uint64_t tm = mask; tm; tm &= tm - 1) {
            const HbArgs& a = hb_launder(a_);   // (re-read per topic: SGPR pressure)
            const int32_t t = __ffsll((long long)tm) - 1;
            // the candidates of every PRUNE of topic t but its own peer: connected
            // peers in t scored >= 0 (a bit per row position, once per topic)
            if constexpr (SPLIT) __syncthreads();                // the last topic's PRUNEs are done with cb
            else wave_lds_sync();
            for (int q0 = SPLIT ? wid * 64 : 0; q0 < deg; q0 += SPLIT ? 64 * WV : 64) {
                const int q = q0 + lane;
                bool c = false;
                if (q < deg) {
                    const uint32_t e = b + (uint32_t)q;
                    c = (a.rstate[e] & GSIM_ES_CONNECTED) && ((a.sub[a.col[e]] >> t) & 1ull) && sc[q] >= 0.0;
                    if (c) pb[q] = px_base(a.seed, key_tick, gobs, (uint32_t)t, purpose, glob(a, a.col[e]));
                }
                const uint64_t bm = __ballot(c);
                if (lane == 0) cb[q0 >> 6] = bm;
            }
            if constexpr (SPLIT) __syncthreads();
            else wave_lds_sync();
            for (int p0 = 0; p0 < deg; p0 += 64) {
                const uint32_t ep_l = b + (uint32_t)(p0 + lane);
                const uint64_t mp = p0 + lane < deg ? smask_of(a.smask, a.col[ep_l]) : 0ull;
                // (a Leave's PRUNE in the same inbox, GSIM_CTL_UNSUB, was listed at the Leave)
                const bool pr = slot_has(mp, t) &&
                                (a.ctl_out[slot_idx(mp, t, a.E, a.rev[ep_l])] & (GSIM_CTL_PX | GSIM_CTL_UNSUB)) == GSIM_CTL_PX;
                for (uint64_t pm = __ballot(pr); pm; pm &= pm - 1) {
                    if constexpr (SPLIT) {
                        if ((turn++ % WV) != wid) continue;
                    }
                    const int pos = p0 + __ffsll((long long)pm) - 1;
                    const uint32_t ep = b + (uint32_t)pos, p = a.col[ep];
                    // a ghost p: its shard holds its score of obs and its row (below)
                    const bool remote = a.pxout && (p < a.olo || p >= a.ohi);
                    if (!remote && a.score[ep] < a.accept_px) continue;   // p's snapshot score of obs (record order)
                    // the PRUNE's candidates (every candidate of t but p) and their keys
                    auto kget = [&](int q) -> uint64_t {
                        return (q != pos && ((cb[q >> 6] >> (q & 63)) & 1ull)) ? px_key(pb[q], (uint32_t)pos, (uint32_t)q)
                                                                                 : ~0ull;
                    };
                    uint32_t n = 0;
                    for (int w = lane; w < (deg + 63) / 64; w += 64) n += (uint32_t)__popcll(cb[w]);
                    n = (uint32_t)wave_sum_u32(n) - (uint32_t)((cb[pos >> 6] >> (pos & 63)) & 1ull);
                    // the keys below a bound that holds ~PrunePeers + 24 of the (uniform)
                    // high words, listed in row order in one pass; the PrunePeers smallest
                    // are then ranked within the list (if it holds them and fits)
                    const uint64_t tau_hi = (int32_t)n <= kPxList || (double)(a.prune_peers + 24) >= (double)n
                                                ? ~0ull
                                                : (uint64_t)((double)(a.prune_peers + 24) / (double)n * 4294967296.0) << 32;
                    uint32_t nl = 0;
                    for (int q0 = 0; q0 < deg; q0 += 64) {
                        const int q = q0 + lane;
                        const uint64_t kv = q < deg ? kget(q) : ~0ull;
                        const bool in = kv != ~0ull && kv < tau_hi;
                        const uint64_t bm = __ballot(in);
                        const uint32_t at = nl + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
                        if (in && at < (uint32_t)kPxList) lst[at] = kv;
                        nl += (uint32_t)__popcll(bm);
                    }
                    wave_lds_sync();
                    const bool listed = nl <= (uint32_t)kPxList && ((int32_t)nl >= a.prune_peers || tau_hi == ~0ull);
                    // exclusive bound: the PrunePeers smallest keys are those below tau
                    uint64_t tau = ~0ull;
                    if (listed) {
                        if ((int32_t)nl > a.prune_peers) {
                            const uint64_t kv = lane < (int)nl ? lst[lane] : ~0ull;
                            uint32_t rank = 0;
                            for (uint32_t j = 0; j < nl; ++j) rank += lst[j] < kv;
                            const uint64_t hit = __ballot(lane < (int)nl && (int32_t)rank == a.prune_peers);
                            tau = (uint64_t)__shfl((long long)kv, __builtin_ctzll(hit), 64);
                        }
                    } else if ((int32_t)n > a.prune_peers) {
                        // the list missed: start from the quantile estimate, then move tau
                        // past one key at a time (as select_smallest)
                        tau = (uint64_t)((double)a.prune_peers / (double)n * 4294967296.0) << 32;
                        int32_t c = 0;
                        for (int q0 = 0; q0 < deg; q0 += 64) {
                            const int q = q0 + lane;
                            c += (int32_t)__popcll(__ballot(q < deg && kget(q) < tau));
                        }
                        while (c > a.prune_peers) {                // drop the largest key below tau
                            uint64_t mx = 0;
                            for (int q0 = 0; q0 < deg; q0 += 64) {
                                const int q = q0 + lane;
                                const uint64_t kv = q < deg ? kget(q) : ~0ull;
                                if (kv < tau && kv >= mx) mx = kv;
                            }
                            mx = wave_max_u64(mx);
                            tau = mx;
                            --c;
                        }
                        while (c < a.prune_peers) {                // add the smallest key at or above tau
                            uint64_t mn = ~0ull;
                            for (int q0 = 0; q0 < deg; q0 += 64) {
                                const int q = q0 + lane;
                                const uint64_t kv = q < deg ? kget(q) : ~0ull;
                                if (kv >= tau && kv < mn) mn = kv;
                            }
                            mn = wave_min_u64(mn);
                            tau = mn + 1;
                            ++c;
                        }
                    }
                    // the list's entries in row order: from the ranked list, else a pass
                    // over the row (lane-strided: entry j of chunk j / 64)
                    const int span = listed ? (int)nl : deg;
                    const uint32_t d = remote ? a.pshard[p] : 0u;
                    const uint64_t hdr = remote ? ((uint64_t)a.xre[ep] | ((uint64_t)t << 32)) : 0ull;
                    const uint32_t rb = a.row_ptr[p], re = a.row_ptr[p + 1];
                    for (int j0 = 0; j0 < span; j0 += 64) {
                        const int j = j0 + lane;
                        int q = -1;
                        if (listed) {
                            if (j < span && lst[j] < tau) q = (int)(uint32_t)lst[j];
                        } else if (j < span && kget(j) < tau) {
                            q = j;
                        }
                        if (remote) {
                            // the PX list to p's shard, which makes handlePrune's checks (k_px_import)
                            const uint64_t bm = __ballot(q >= 0);
                            uint32_t base = 0;
                            if (lane == 0 && bm) base = atomicAdd(&a.pxcnt[d], (uint32_t)__popcll(bm));
                            base = (uint32_t)__shfl((int)base, 0, 64);
                            if (q < 0) continue;
                            const uint32_t k = base + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
                            const uint64_t gx = glob(a, a.col[b + (uint32_t)q]);
                            if ((int64_t)k < a.pxcap) a.pxout[(int64_t)d * a.pxcap + k] = hdr | (gx << 38);
                            else atomicOr(&a.pxcnt[a.pxK], 1u);
                            continue;
                        }
                        if (q < 0) continue;
                        const uint32_t x = a.col[b + (uint32_t)q];
                        uint32_t lo = rb, hi = re;                 // p's row is sorted: its edge to x
                        while (lo < hi) {
                            const uint32_t mid = lo + ((hi - lo) >> 1);
                            if (a.col[mid] < x) lo = mid + 1; else hi = mid;
                        }
                        // pxConnect skips peers it is connected to
                        if (lo < re && a.col[lo] == x && !(a.rstate[lo] & GSIM_ES_CONNECTED)) a.pxm[lo] = 1;
                    }
                    wave_lds_sync();                               // lst is rewritten by the next PRUNE
                }
            }
        }
        if constexpr (SPLIT) __syncthreads();                    // sc is rewritten by the next observer
    }
}

// makePrune's PX lists of every observer that sent PX PRUNEs: rows of at most
// 256 connections a wave each (4 observers per block), hub rows (257-1024,
// 1025-4096) a block of 4 waves each sharing the observer's scores and taking
// its PRUNEs in turn (a hub's GRAFT replies are many: one wave made c5's hub
// pass 20 ms per tick).
constexpr int kPxSmall = 256;
static void launch_px_emit(gsim_handle* h, const HbArgs& a, int live, uint32_t key_tick, uint32_t purpose)
{
    const Extra* x = h->x;
    const int64_t nown = h->ohi() - h->olo();
    hipLaunchKernelGGL((k_px_emit<kPxSmall, 4>), dim3((uint32_t)std::min<int64_t>(std::max<int64_t>((nown + 3) / 4, 1), 65536)),
                       dim3(256), 0, h->stream, a, live, key_tick, purpose, (const uint32_t*)nullptr, (int64_t)0);
    if (!x->d_rows) return;                      // one class of rows <= 16: no hub
    const uint32_t* rh = x->d_rows + x->n16 + x->n32 + x->n64 + x->nh256;
    if (x->nh1024)
        hipLaunchKernelGGL((k_px_emit<kPxRow, 4, true>), dim3((uint32_t)std::min<int64_t>(x->nh1024, 65536)), dim3(256),
                           0, h->stream, a, live, key_tick, purpose, rh, x->nh1024);
    if (x->nh4096)
        hipLaunchKernelGGL((k_px_emit<4 * kPxRow, 4, true>), dim3((uint32_t)std::min<int64_t>(x->nh4096, 65536)),
                           dim3(256), 0, h->stream, a, live, key_tick, purpose, rh + x->nh1024, x->nh4096);
    if (x->nh8192)   // (scores, candidate bits and draws of 8192 positions: 97 KB of LDS)
        hipLaunchKernelGGL((k_px_emit<kGiantRow, 4, true>), dim3((uint32_t)std::min<int64_t>(x->nh8192, 65536)),
                           dim3(256), 0, h->stream, a, live, key_tick, purpose, rh + x->nh1024 + x->nh4096, x->nh8192);
}

// Connection attempts to connections (the connector, gossipsub.go:941-973):
// each marked pair once (from its lower end), dialled by the peer that asked
// (the lower id when both did); pairs already connected are skipped.  Out:
// pxc[0] = count, then per connection (dialer's edge, peer's edge).
__global__ __launch_bounds__(256) void k_px_collect(const uint32_t* owner, const uint32_t* col, const uint32_t* rev,
                                                    const uint8_t* rstate, uint8_t* pxm, int64_t E, uint32_t* pxc)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) {
        const uint32_t u = owner[e], v = col[e], r = rev[e];
        if (u > v) continue;
        const uint8_t x = pxm[e], y = pxm[r];
        if (!(x | y)) continue;
        pxm[e] = 0;
        pxm[r] = 0;
        if (rstate[e] & GSIM_ES_CONNECTED) continue;
        const uint32_t k = atomicAdd(pxc, 1u);
        pxc[1 + 2 * k] = x ? (uint32_t)e : r;
        pxc[2 + 2 * k] = x ? r : (uint32_t)e;
    }
}

__global__ __launch_bounds__(256) void k_px_pairs(const uint32_t* pxc, uint32_t n, const uint32_t* owner,
                                                  const uint32_t* col, uint32_t* out)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t ed = pxc[1 + 2 * k];
    out[2 * k] = owner[ed];
    out[2 * k + 1] = col[ed];
}

__global__ __launch_bounds__(256) void k_px_outbound(const uint32_t* pxc, uint32_t n, uint8_t* outbound)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    outbound[pxc[1 + 2 * k]] = 1;          // gs.outbound: the dialer's side (gossipsub.go:532-551)
    outbound[pxc[2 + 2 * k]] = 0;
}

// A shard's end of a remote pruner's PX lists (entries of k_px_emit's remote
// path): handlePrune's acceptPXThreshold on the pruned peer's snapshot score
// of the pruner (its record at the cross edge's index r here), then
// pxConnect's attempt to every listed peer with a known address (an edge of
// the pruned peer's row) it is not connected to.
__global__ __launch_bounds__(256) void k_px_import(const uint64_t* in, int64_t n, const double* score,
                                                   const uint32_t* col, const uint32_t* row_ptr, const uint8_t* rstate,
                                                   const uint32_t* g2l, double accept_px, uint8_t* pxm)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        const uint64_t v = in[k];
        const uint32_t r = (uint32_t)v;
        if (score[r] < accept_px) continue;
        const uint32_t p = col[r], x = g2l ? g2l[(uint32_t)(v >> 38)] : (uint32_t)(v >> 38);
        if (x == 0xFFFFFFFFu) continue;                      // not a neighbour of p
        uint32_t lo = row_ptr[p], hi = row_ptr[p + 1];
        const uint32_t pe = hi;
        while (lo < hi) {
            const uint32_t mid = lo + ((hi - lo) >> 1);
            if (col[mid] < x) lo = mid + 1; else hi = mid;
        }
        if (lo < pe && col[lo] == x && !(rstate[lo] & GSIM_ES_CONNECTED)) pxm[lo] = 1;
    }
}

// A shard's connection attempts: every marked owned-row edge (p asked for x),
// as global (asker | peer << 32); the marks are cleared.
__global__ __launch_bounds__(256) void k_px_asks(const uint32_t* owner, const uint32_t* col, const uint8_t* rstate,
                                                 const uint32_t* gid, uint8_t* pxm, int64_t e_lo, int64_t e_hi,
                                                 uint64_t* out, uint32_t* cnt, int64_t cap)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = e_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e_hi; e += stride) {
        if (!pxm[e]) continue;
        pxm[e] = 0;
        if (rstate[e] & GSIM_ES_CONNECTED) continue;
        const uint32_t k = atomicAdd(cnt, 1u);
        if ((int64_t)k < cap) out[k] = (uint64_t)gid[owner[e]] | ((uint64_t)gid[col[e]] << 32);
    }
}

// The connector's (dialer | peer << 32) global pairs: gs.outbound on this
// shard's owned ends (the dialer's side outbound, the peer's not).
__global__ __launch_bounds__(256) void k_px_outbound_pairs(const uint64_t* pairs, int64_t n, const uint32_t* g2l,
                                                           const uint32_t* row_ptr, const uint32_t* col, uint32_t olo,
                                                           uint32_t ohi, uint8_t* outbound)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < 2 * n; k += stride) {
        const uint64_t v = pairs[k >> 1];
        const bool dial = !(k & 1);
        const uint32_t a_ = g2l[dial ? (uint32_t)v : (uint32_t)(v >> 32)], b_ = g2l[dial ? (uint32_t)(v >> 32) : (uint32_t)v];
        if (a_ == 0xFFFFFFFFu || b_ == 0xFFFFFFFFu || a_ < olo || a_ >= ohi) continue;
        uint32_t lo = row_ptr[a_], hi = row_ptr[a_ + 1];
        const uint32_t pe = hi;
        while (lo < hi) {
            const uint32_t mid = lo + ((hi - lo) >> 1);
            if (col[mid] < b_) lo = mid + 1; else hi = mid;
        }
        if (lo < pe && col[lo] == b_) outbound[lo] = dial ? 1 : 0;
    }
}

bool px_enabled(const gsim_handle* h) { return h->x && h->x->d_pxo; }

void row_classes(gsim_handle* h, RowClasses* rc)
{
    const Extra* x = h->x;
    if (!x) { *rc = RowClasses{nullptr, 0, 0, h->ohi() - h->olo(), 0}; return; }
    *rc = RowClasses{x->d_rows, x->n16, x->n32, x->n64, x->nh256 + x->nh1024 + x->nh4096 + x->nh8192};
}

int px_import(gsim_handle* h, const uint64_t* d_in, int64_t n)
{
    if (n <= 0 || !h->x || !h->x->d_pxm) return GSIM_OK;
    hipLaunchKernelGGL(k_px_import, dim3((uint32_t)std::min<int64_t>((n + 255) / 256, 16384)), dim3(256), 0, h->stream,
                       d_in, n, (const double*)h->d_score, (const uint32_t*)h->d_col, (const uint32_t*)h->d_row_ptr,
                       (const uint8_t*)h->d_rstate, (const uint32_t*)h->sh->d_g2l, h->th.accept_px_threshold,
                       h->x->d_pxm);
    return hip_check(h, hipGetLastError(), "k_px_import");
}

// Leave's PX lists (Extra::d_pxl) to their pruned peers (local to this
// handle): handlePrune's acceptPXThreshold on the snapshot, pxConnect's
// attempts (k_px_import); the lists are consumed.  g2l: a shard's global ->
// local ids (nullptr: a single engine).
int px_leave_import(gsim_handle* h, const uint32_t* g2l)
{
    if (!h->x || !h->x->d_pxl_n) return GSIM_OK;
    uint32_t n[2] = {0, 0};
    hipError_t e = hipMemcpyAsync(n, h->x->d_pxl_n, sizeof(n), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "Leave PX count");
    if (n[1]) { h->err = "Leave PX list overflow"; return GSIM_ERANGE; }
    if (!n[0]) return GSIM_OK;
    hipLaunchKernelGGL(k_px_import, dim3((uint32_t)std::min<int64_t>((n[0] + 255) / 256, 16384)), dim3(256), 0,
                       h->stream, (const uint64_t*)h->x->d_pxl, (int64_t)n[0], (const double*)h->d_score,
                       (const uint32_t*)h->d_col, (const uint32_t*)h->d_row_ptr, (const uint8_t*)h->d_rstate, g2l,
                       h->th.accept_px_threshold, h->x->d_pxm);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemsetAsync(h->x->d_pxl_n, 0, sizeof(n), h->stream);
    return hip_check(h, e, "k_px_import (Leave)");
}

bool deliver_wire_px(gsim_handle* h, WirePx* w)
{
    if (!h->x || !h->x->d_pxo) return false;
    uint32_t n[2] = {0, 0};
    if (hipMemcpyAsync(n, h->x->d_pxl_n, sizeof(n), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess)
        n[0] = 0;
    *w = WirePx{h->x->d_pxs, h->x->seed, h->x->d_pxl, h->x->d_pxl_tick, n[0]};
    return true;
}

int px_asks(gsim_handle* h, uint64_t* d_out, uint32_t* d_cnt, int64_t cap)
{
    hipError_t e = hipMemsetAsync(d_cnt, 0, sizeof(uint32_t), h->stream);
    if (e != hipSuccess || !h->x || !h->x->d_pxm) return hip_check(h, e, "px asks");
    const int64_t lo = h->sh->own_e_lo, hi = h->sh->own_e_hi;
    hipLaunchKernelGGL(k_px_asks, dim3((uint32_t)std::min<int64_t>((hi - lo + 255) / 256 + 1, 16384)), dim3(256), 0,
                       h->stream, (const uint32_t*)h->d_owner, (const uint32_t*)h->d_col, (const uint8_t*)h->d_rstate,
                       (const uint32_t*)h->sh->d_gid, h->x->d_pxm, lo, hi, d_out, d_cnt, cap);
    return hip_check(h, hipGetLastError(), "k_px_asks");
}

int px_mark_outbound(gsim_handle* h, const uint64_t* d_pairs, int64_t n)
{
    if (n <= 0) return GSIM_OK;
    hipLaunchKernelGGL(k_px_outbound_pairs, dim3((uint32_t)std::min<int64_t>((2 * n + 255) / 256, 16384)), dim3(256),
                       0, h->stream, d_pairs, n, (const uint32_t*)h->sh->d_g2l, (const uint32_t*)h->d_row_ptr,
                       (const uint32_t*)h->d_col, (uint32_t)h->olo(), (uint32_t)h->ohi(), h->d_outbound);
    return hip_check(h, hipGetLastError(), "k_px_outbound_pairs");
}

// inspectScoresExtended (score.go:472-500) for the connections e of
// [e_lo, e_hi): the live score and its components.
__global__ __launch_bounds__(256) void k_snapshot(HbArgs a, int64_t e_lo, int64_t e_hi, gsim_peer_score_snapshot* ps,
                                                  gsim_topic_score_snapshot* ts)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = e_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e_hi; e += stride) {
        const int64_t x = e - e_lo;
        const uint32_t col = a.col[e], rv = a.rev[e];
        const bool tracked = (a.estate[rv] & GSIM_ES_TRACKED) != 0;
        gsim_peer_score_snapshot p{};
        p.observer = glob(a, a.col[rv]);
        p.peer = glob(a, col);
        p.tracked = tracked ? 1 : 0;
        if (tracked) {
            p.score = score_of_record(a, rv, col);
            p.app_specific_score = a.p5[col];
            p.ip_colocation_factor = a.p6[rv];
            p.behaviour_penalty = a.bp[rv];
        }
        ps[x] = p;
        const uint64_t mj = smask_of(a.smask, col);
        for (int32_t t = 0; t < a.T; ++t) {
            const int64_t i = slot_idx(mj, t, a.E, rv);
            gsim_topic_score_snapshot q{};
            if (tracked && slot_has(mj, t)) {
                const uint8_t fl = a.tflags[i];
                q.time_in_mesh_ns = !(fl & GSIM_TF_IN_MESH) ? 0
                                    : lazy_mtime(a.mt_lazy && (a.estate[rv] & GSIM_ES_CONNECTED), a.mt_R, a.graft[i],
                                                 a.mtime[i]);
                q.first_message_deliveries = a.first[i];
                q.mesh_message_deliveries =
                    apply_incs(a.meshd[i], a.mcnt[i], const_tp(a.tp)[t].mesh_message_deliveries_cap);
                q.invalid_message_deliveries = a.invalid[i];
            }
            ts[x * a.T + t] = q;
        }
    }
}

// ---------------------------------------------------------------------------
// Connection churn between ticks (handleDeadPeers pubsub.go:711-759, the
// new-peer case of processLoop pubsub.go:575-595): both endpoints of each
// listed connection run the router's RemovePeer / AddPeer
// (gossipsub.go:525-567) and the score tracer's (score.go:595-644).

struct ChurnArgs {
    const uint32_t* edges;     // [2*count] the observer's edge of each (pair, direction)
    int32_t n2;
    int32_t up;
    int64_t retain;            // PeerScoreParams.RetainScore
    uint8_t *estate, *rstate, *pen;
    int64_t* expire;
    double *first, *invalid;
    int32_t skip_unjoined;     // records of topics their observer did not join are zero (engine.hip)
    uint8_t* p6row;            // [N] rows whose P6 must be re-derived (engine.hip launch_ip_colocation)
};

// The observer's edge to the other end of each (pair, direction), by binary
// search in the observer's sorted row; *bad = lowest pair that is not a
// connection.
// Join / Leave (gossipsub.go:1047-1124) of the (peer, topic) pairs in order:
// one thread, because each change is seen by the later ones (the topic peers
// of a Join include the peers that joined before it), as in the oracle's
// orc_set_subscriptions.  Rare and between ticks.
__device__ __forceinline__ bool sub_topic_peer(const HbArgs& a, uint64_t* sub, uint32_t e, int32_t t)
{
    return (a.rstate[e] & GSIM_ES_CONNECTED) && ((sub[a.col[e]] >> t) & 1ull);
}

// Leave's sendPrune(p, topic, true) -> makePrune(p, topic, gs.doPX, true)
// (gossipsub.go:1118, 1132-1133, 1866-1906): the PX list of the PRUNE at row
// edge ep, getPeers(topic, PrunePeers, xp != p && Score(xp) >= 0) with the
// live scores after the Leave's Prunes so far (sc[], the observer's row in
// pxs), the PrunePeers smallest keys in key order.  Kept for the connector
// (the pruned peer's handlePrune runs with the tick's control: its snapshot
// after the next refresh) and the wire encoder; a pruned peer of another
// shard gets its list through the group's PX exchange, as k_px_emit's.
__device__ void px_leave_list(const HbArgs& a, const uint64_t* sub, uint32_t obs, uint32_t b, uint32_t en, uint32_t ep,
                              int32_t t)
{
    const double* sc = a.pxs;
    const uint32_t gobs = glob(a, obs);
    const uint32_t p = a.col[ep];
    const bool remote = a.pxout && (p < a.olo || p >= a.ohi);
    uint64_t last = 0;
    for (int k = 0; k < a.prune_peers; ++k) {
        uint64_t best = ~0ull;
        uint32_t bx = 0xFFFFFFFFu;
        for (uint32_t e = b; e < en; ++e) {
            if (e == ep || !sub_topic_peer(a, const_cast<uint64_t*>(sub), e, t) || sc[e] < 0.0) continue;
            const uint64_t key = px_key(px_base(a.seed, (uint32_t)a.tick, gobs, (uint32_t)t, P_PX_LEAVE, glob(a, a.col[e])),
                                        ep - b, e - b);
            if ((k > 0 && key <= last) || key >= best) continue;
            best = key;
            bx = e;
        }
        if (bx == 0xFFFFFFFFu) break;
        last = best;
        const uint64_t gx = glob(a, a.col[bx]);
        if (remote) {
            const uint32_t d = a.pshard[p];
            const uint32_t q = atomicAdd(&a.pxcnt[d], 1u);
            if ((int64_t)q < a.pxcap) a.pxout[(int64_t)d * a.pxcap + q] = (uint64_t)a.xre[ep] | ((uint64_t)t << 32) | (gx << 38);
            else atomicOr(&a.pxcnt[a.pxK], 1u);
        } else {
            const uint32_t q = a.pxl_n[0]++;
            if ((int64_t)q < a.pxl_cap) {
                a.pxl[q] = (uint64_t)ep | ((uint64_t)t << 32) | (gx << 38);
                a.pxl_tick[q] = (uint32_t)a.tick;
            } else {
                a.pxl_n[1] = 1;
            }
        }
    }
}

// Σ row lengths of the pairs' peers (Leave's PX list entries need at most
// PrunePeers per connection of a leaving peer)
__global__ void k_pair_degrees(const uint32_t* row_ptr, const uint32_t* pairs, int32_t count, unsigned long long* out)
{
    unsigned long long s = 0;
    for (int32_t q = threadIdx.x; q < count; q += blockDim.x) s += row_ptr[pairs[2 * q] + 1] - row_ptr[pairs[2 * q]];
    atomicAdd(out, s);
}

__global__ void k_subscribe(HbArgs a, uint64_t* sub, const uint32_t* pairs, int32_t count, int32_t join)
{
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    for (int32_t q = 0; q < count; ++q) {
        const uint32_t p = pairs[2 * q];
        const int32_t t = (int32_t)pairs[2 * q + 1];
        const uint64_t bit = 1ull << t;
        const uint32_t b = a.row_ptr[p], en = a.row_ptr[p + 1];
        const uint64_t mi = smask_of(a.smask, p);           // p's router state (its slots: gsim_set_subscriptions grew them)
        const uint32_t gp_ = glob(a, p);
        auto mf = [&](uint32_t e) -> uint8_t& { return a.mflags[slot_idx(mi, t, a.E, e)]; };
        auto bo = [&](uint32_t e) -> int64_t& { return a.backoff[slot_idx(mi, t, a.E, e)]; };
        auto send = [&](uint32_t e, uint8_t bits) {
            const uint32_t c = a.col[e];
            const uint64_t mq = smask_of(a.smask, c);
            if (!slot_has(mq, t)) return;
            const int64_t r = slot_idx(mq, t, a.E, a.rev[e]);   // the receiver's inbox entry
            a.ctl_out[r] = (uint8_t)(a.ctl_out[r] | bits);
            atomicOr(reinterpret_cast<unsigned long long*>(a.cany_out + c), bit);
        };
        const ctp_t tp = const_tp(a.tp) + t;
        // a shard: a ghost's announcement only (its own shard runs its router)
        const bool own = p >= a.olo && p < a.ohi;
        if (join) {
            if (sub[p] & bit) continue;                      // gs.mesh[topic] exists
            sub[p] |= bit;                                   // the announcement
            if (!own) continue;
            if (a.tr.on(p)) a.tr.push(a.now, 0, p, p, t, GSIM_TRACE_JOIN, 0);
            // getPeers: the `count` candidates with the smallest keys, in key order
            auto pick = [&](int count, bool more) {
                uint64_t last = 0;
                bool first_pick = true;
                for (int k = 0; k < count; ++k) {
                    uint64_t best = ~0ull;
                    uint32_t be = 0xFFFFFFFFu;
                    for (uint32_t e = b; e < en; ++e) {
                        if (!sub_topic_peer(a, sub, e, t)) continue;
                        // the live Score(p) (gossipsub.go:1076, 1091): deliveries since the
                        // last refresh count, as for emitGossip's candidates
                        if (a.direct[e] || bo(e) != 0 || score_of_record(a, a.rev[e], a.col[e]) < 0.0) continue;
                        if (more && (mf(e) & GSIM_TF_FANOUT)) continue;
                        const uint64_t key = hb_key(a, gp_, t, P_JOIN, glob(a, a.col[e]), e - b);
                        if ((!first_pick && key <= last) || key >= best) continue;
                        best = key;
                        be = e;
                    }
                    if (be == 0xFFFFFFFFu) break;
                    last = best;
                    first_pick = false;
                    mf(be) |= more ? GSIM_TF_FANOUT : GSIM_TF_MESH;
                }
            };
            if ((a.fan_topics[p] >> t) & 1ull) {
                int have = 0;
                for (uint32_t e = b; e < en; ++e) {
                    if (!(mf(e) & GSIM_TF_FANOUT)) continue;
                    if (score_of_record(a, a.rev[e], a.col[e]) < 0.0 || bo(e) != 0)   // live Score (1063)
                        mf(e) &= (uint8_t)~GSIM_TF_FANOUT;
                    else ++have;
                }
                if (have < a.D) pick(a.D - have, true);
                for (uint32_t e = b; e < en; ++e)
                    if (mf(e) & GSIM_TF_FANOUT) mf(e) = (uint8_t)((mf(e) & ~GSIM_TF_FANOUT) | GSIM_TF_MESH);
                a.fan_topics[p] &= ~bit;                     // delete(gs.fanout, topic), delete(gs.lastpub, topic)
                a.lastpub[(int64_t)p * a.T + t] = 0;
            } else {
                pick(a.D, false);
            }
            for (uint32_t e = b; e < en; ++e) {
                if (!(mf(e) & GSIM_TF_MESH)) continue;
                if (a.tr.on(p)) a.tr.push(a.now, 0, p, a.col[e], t, GSIM_TRACE_GRAFT, 0);   // tracer.Graft
                const uint32_t rv = a.rev[e];
                ScoreFlags sf;
                sf.at(smask_of(a.smask, a.col[e]), t, a.E, rv);
                stats_graft(a, (a.estate[rv] & GSIM_ES_TRACKED) != 0, tp->scored != 0, sf);
                sf.store(a);
                send(e, GSIM_CTL_GRAFT);
            }
        } else {
            if (!(sub[p] & bit)) continue;                   // no mesh for the topic
            sub[p] &= ~bit;
            if (!own) continue;
            if (a.tr.on(p)) a.tr.push(a.now, 0, p, p, t, GSIM_TRACE_LEAVE, 0);
            // emitGossip no longer runs for the topic (unless as a fanout): its
            // last IHAVE targets must not be advertised to again
            if (a.gsel)
                for (uint32_t e = b; e < en; ++e) a.gsel[slot_idx(mi, t, a.E, e)] = 0;
            if (a.do_px)     // the live scores makePrune's PX filter reads (updated per Prune below)
                for (uint32_t e = b; e < en; ++e) a.pxs[e] = score_of_record(a, a.rev[e], a.col[e]);
            for (uint32_t e = b; e < en; ++e) {
                if (!(mf(e) & GSIM_TF_MESH)) continue;
                if (a.tr.on(p)) a.tr.push(a.now, 0, p, a.col[e], t, GSIM_TRACE_PRUNE, 0);   // tracer.Prune
                const uint32_t rv = a.rev[e];
                ScoreFlags sf;
                sf.at(smask_of(a.smask, a.col[e]), t, a.E, rv);
                stats_prune(a, (a.estate[rv] & GSIM_ES_TRACKED) != 0, tp->scored != 0,
                            tp->mesh_message_deliveries_threshold, tp->mesh_message_deliveries_cap, sf);
                sf.store(a);
                mf(e) &= (uint8_t)~GSIM_TF_MESH;
                send(e, (uint8_t)(GSIM_CTL_PRUNE | GSIM_CTL_UNSUB | (a.do_px ? GSIM_CTL_PX : 0)));
                const int64_t ex = a.now + a.unsub_backoff;   // addBackoff(p, topic, isUnsubscribe)
                if (bo(e) < ex) bo(e) = ex;
                if (a.do_px) {
                    a.pxs[e] = score_of_record(a, rv, a.col[e]);   // tracer.Prune changed this record
                    px_leave_list(a, sub, p, b, en, e, t);
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_churn_find(const uint32_t* row_ptr, const uint32_t* col, int64_t N,
                                                    const uint32_t* pairs, int32_t n2, uint32_t* edges,
                                                    uint32_t* bad, uint32_t* mark)
{
    const int32_t q = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= n2) return;
    const uint32_t o = pairs[(q & ~1) + (q & 1)], p = pairs[(q & ~1) + 1 - (q & 1)];
    uint32_t e = 0xFFFFFFFFu;
    if (o < N && p < N) {
        uint32_t lo = row_ptr[o], hi = row_ptr[o + 1];
        const uint32_t end = hi;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (col[mid] < p) lo = mid + 1; else hi = mid;
        }
        if (lo < end && col[lo] == p) e = lo;
    }
    edges[q] = e;
    if (e == 0xFFFFFFFFu) {
        atomicMin(bad, (uint32_t)(q >> 1));
    } else if (o < p) {
        // the connection's lower-to-higher edge, marked once per listing: a
        // second listing (in either order) finds the mark set
        const uint32_t bit = 1u << (e & 31);
        if (atomicOr(mark + (e >> 5), bit) & bit) atomicMin(bad + 1, (uint32_t)(q >> 1));
    }
}

// Clears the marks k_churn_find set (the bitmap is zero between calls).
__global__ __launch_bounds__(256) void k_churn_unmark(const uint32_t* pairs, const uint32_t* edges, int32_t n2,
                                                      uint32_t* mark)
{
    const int32_t q = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= n2) return;
    const uint32_t o = pairs[(q & ~1) + (q & 1)], p = pairs[(q & ~1) + 1 - (q & 1)];
    const uint32_t e = edges[q];
    if (e != 0xFFFFFFFFu && o < p) atomicAnd(mark + (e >> 5), ~(1u << (e & 31)));
}

// Fresh (or dropped) score record r: an empty peerStats.
// joined: topics whose records may be non-zero (within the row owner's slots mj)
__device__ void churn_reset_record(const HbArgs& a, const ChurnArgs& c, uint32_t r, uint64_t joined, uint64_t mj)
{
    a.bp[r] = 0.0;
    c.expire[r] = 0;
    c.pen[r] = 0;
    for (int32_t t = 0; t < a.T; ++t) {
        if (!((joined >> t) & 1ull)) continue;   // already zero
        const int64_t i = slot_idx(mj, t, a.E, r);
        c.first[i] = 0.0; a.meshd[i] = 0.0; a.fail[i] = 0.0; c.invalid[i] = 0.0;
        a.graft[i] = 0; a.mtime[i] = 0;
        a.tflags[i] = 0;
        if (GSIM_CHURN_MCNT) a.mcnt[i] = 0;       // pending deliveries of the dropped record
    }
}

// One thread per (connection, direction): the observer owning edge e, about
// neighbour col[e]; the observer's record of it sits at rev[e].
__global__ __launch_bounds__(256) void k_churn_apply(HbArgs a, ChurnArgs c)
{
    const int32_t q = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= c.n2) return;
    const uint32_t e = c.edges[q];
    const uint32_t r = a.rev[e];
    if (a.col[r] < a.olo || a.col[r] >= a.ohi) return;   // the other shard handles a ghost observer's side
    if (c.p6row) c.p6row[a.col[r]] = 1;                   // the observer's tracked set may change: P6 of its row
    if (a.tr.on(a.col[r]))                                 // tracer.AddPeer / RemovePeer (trace.go:196-248)
        a.tr.push(a.now, 0, a.col[r], a.col[e], -1, c.up ? GSIM_TRACE_ADD_PEER : GSIM_TRACE_REMOVE_PEER, 0);
    // the observer's (col[r]) joined topics while unjoined records are known zero:
    // a store to them would write the value already there.  Random 1-8 B stores
    // are the churn's bound, so the router planes below are also stored only
    // where they change.
    // topic slots: the records r sit in the neighbour's row (mj), the router
    // state e in the observer's (mi)
    const uint64_t mj = smask_of(a.smask, a.col[e]), mi = smask_of(a.smask, a.col[r]);
    const uint64_t joined = (c.skip_unjoined ? a.sub[a.col[r]] : ~0ull) & mj;
    if (c.up) {
        // AddPeer: connected; a retained record comes back as it is
        c.rstate[e] = (uint8_t)(c.rstate[e] | GSIM_ES_CONNECTED);
        if (!(c.estate[r] & GSIM_ES_TRACKED)) churn_reset_record(a, c, r, joined, mj);
        c.estate[r] = GSIM_ES_TRACKED | GSIM_ES_CONNECTED;
        return;
    }
    // router RemovePeer: out of every mesh without PRUNE, pending control dropped
    for (int32_t t = 0; t < a.T; ++t) {
        if (!slot_has(mi, t)) continue;
        const int64_t i = slot_idx(mi, t, a.E, e);
        const uint8_t mf = a.mflags[i], ci = a.ctl_in[i], co = a.ctl_out[i];
        const uint8_t nm = (uint8_t)(mf & ~(GSIM_TF_MESH | GSIM_TF_FANOUT));
        if (nm != mf) a.mflags[i] = nm;
        if (ci) a.ctl_in[i] = 0;
        if (co) a.ctl_out[i] = 0;
    }
    c.rstate[e] = (uint8_t)(c.rstate[e] & ~GSIM_ES_CONNECTED);
    // peerScore.RemovePeer: positive scores are dropped, the rest retained
    if (!(c.estate[r] & GSIM_ES_TRACKED)) return;
    if (score_of_record(a, r, a.col[e]) > 0) {
        churn_reset_record(a, c, r, joined, mj);
        c.estate[r] = 0;
        return;
    }
    for (int32_t t = 0; t < a.T; ++t) {
        const ctp_t tp = const_tp(a.tp) + t;
        if (!tp->scored || !((joined >> t) & 1ull)) continue;
        const int64_t i = slot_idx(mj, t, a.E, r);
        c.first[i] = 0.0;
        const uint8_t fl = a.tflags[i];
        const double thr = tp->mesh_message_deliveries_threshold;
        double md = a.meshd[i];
        if (GSIM_CHURN_MCNT) {
            // the record's pending deliveries are part of the counter (RemovePeer's P3b
            // reads it): applied here, not by a pass over every record first
            const uint8_t pc = a.mcnt[i];
            if (pc) {
                md = apply_incs(md, pc, tp->mesh_message_deliveries_cap);
                a.meshd[i] = md;
                a.mcnt[i] = 0;
            }
        }
        if ((fl & GSIM_TF_IN_MESH) && (fl & GSIM_TF_ACTIVE) && md < thr) {
            const double deficit = thr - md;
            a.fail[i] = a.fail[i] + deficit * deficit;
        }
        if (fl & GSIM_TF_IN_MESH) a.mtime[i] = 0;   // meshTime outside the mesh is 0
        a.tflags[i] = (uint8_t)(fl & ~GSIM_TF_IN_MESH);
    }
    c.estate[r] = GSIM_ES_TRACKED;
    c.expire[r] = a.now + c.retain;
}

// Publish's fanout branch (gossipsub.go:1011-1028), one wave per published
// message whose origin has not joined the topic: with no fanout peers yet,
// getPeers(topic, D, score >= publishThreshold) becomes the fanout (Philox
// counter word 0 = the round, a.tick); then lastpub = now.  Of several
// messages of one (origin, topic) in a batch the first does the selection
// (the others would find the fanout non-empty).
template <class Grp>
__device__ __forceinline__ void fanout_publish_one(const HbArgs& a, Grp& g, const gsim_msg* pub, int32_t k)
{
    constexpr int V = Grp::V;
    const int gl0 = g.pos(0);
    const uint32_t o = pub[k].origin;
    const int32_t t = (int32_t)pub[k].topic;
    bool dup[V];
#pragma unroll
    for (int v = 0; v < V; ++v) dup[v] = false;
    for (int32_t q = gl0; q < k; q += g.span() / V) dup[0] |= pub[q].origin == o && (int32_t)pub[q].topic == t;
    if (g.any(dup)) return;
    const uint32_t b = a.row_ptr[o];
    const int deg = (int)(a.row_ptr[o + 1] - b);
    const uint64_t mo = smask_of(a.smask, o);      // gsim_publish gave the origin a slot for t
    if (!slot_has(mo, t)) return;                  // group-uniform
    bool valid[V], isf[V];
    uint32_t e[V];
    int64_t i[V];
    uint8_t fl[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        valid[v] = g.pos(v) < deg;
        e[v] = b + (uint32_t)g.pos(v);
        i[v] = slot_idx(mo, t, a.E, e[v]);
        fl[v] = valid[v] ? a.mflags[i[v]] : 0;
        isf[v] = (fl[v] & GSIM_TF_FANOUT) != 0;
    }
    const bool have = ((a.fan_topics[o] >> t) & 1ull) && g.any(isf);
    if (!have) {
        uint32_t gcol[V];
        bool cand[V], sel[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const uint32_t col = valid[v] ? a.col[e[v]] : 0u;
            const bool conn = valid[v] && (a.rstate[e[v]] & GSIM_ES_CONNECTED);
            const bool tpeer = conn && ((a.sub[col] >> t) & 1ull);
            const double S = valid[v] ? a.score[a.rev[e[v]]] : 0.0;
            cand[v] = tpeer && !isf[v] && !(valid[v] && a.direct[e[v]]) && S >= a.pub_thr;
            gcol[v] = valid[v] ? glob(a, col) : 0u;
        }
        g.select(a, cand, a.D, glob(a, o), t, P_FANOUT_NEW, gcol, sel);
#pragma unroll
        for (int v = 0; v < V; ++v)
            if (valid[v] && sel[v]) a.mflags[i[v]] = (uint8_t)(fl[v] | GSIM_TF_FANOUT);
        const bool any = g.any(sel);
        if (gl0 == 0 && any) atomicOr(reinterpret_cast<unsigned long long*>(a.fan_topics + o), 1ull << t);
    }
    if (gl0 == 0) a.lastpub[(int64_t)o * a.T + t] = a.now;
}

__device__ __forceinline__ bool fanout_publisher(const HbArgs& a, const gsim_msg* pub, int32_t k)
{
    const uint32_t o = pub[k].origin;
    if (o < a.olo || o >= a.ohi) return false;                // published on another shard
    return !((a.sub[o] >> pub[k].topic) & 1ull);               // joined: it publishes to its mesh
}

__global__ __launch_bounds__(256) void k_fanout_publish(HbArgs a, const gsim_msg* pub, int32_t count)
{
    const int32_t k = (int32_t)blockIdx.x * 4 + (int32_t)(threadIdx.x >> 6);
    if (k >= count || !fanout_publisher(a, pub, k)) return;  // wave-uniform
    const uint32_t o = pub[k].origin;
    if (a.row_ptr[o + 1] - a.row_ptr[o] > 64u) return;        // a hub: k_fanout_publish_hub
    WaveGroup<64> g(threadIdx.x & 63);
    fanout_publish_one(a, g, pub, k);
}

// origins with rows of lo+1 .. B·V connections
template <int B, int V>
__global__ __launch_bounds__(B) void k_fanout_publish_hub(HbArgs a, const gsim_msg* pub, int32_t count, uint32_t lo)
{
    __shared__ typename BlockGroup<B, V>::Shared sh;
    const int32_t k = (int32_t)blockIdx.x;
    if (k >= count || !fanout_publisher(a, pub, k)) return;  // block-uniform
    const uint32_t o = pub[k].origin, d = a.row_ptr[o + 1] - a.row_ptr[o];
    if (d <= lo || d > (uint32_t)(B * V)) return;
    BlockGroup<B, V> g(&sh);
    fanout_publish_one(a, g, pub, k);
}

// ... origins with rows of lo+1 .. B*V connections, group state in global
// scratch: the grid strides over the batch (one scratch slice per block)
template <int B, int V>
__global__ __launch_bounds__(B) void k_fanout_publish_hub_g(HbArgs a, const gsim_msg* pub, int32_t count, uint32_t lo,
                                                            void* scratch)
{
    using S = typename BlockGroup<B, V>::Shared;
    BlockGroup<B, V> g(reinterpret_cast<S*>(scratch) + blockIdx.x);
    for (int32_t k = (int32_t)blockIdx.x; k < count; k += (int32_t)gridDim.x) {
        if (!fanout_publisher(a, pub, k)) continue;      // block-uniform
        const uint32_t o = pub[k].origin, d = a.row_ptr[o + 1] - a.row_ptr[o];
        if (d <= lo || d > (uint32_t)(B * V)) continue;
        fanout_publish_one(a, g, pub, k);
    }
}

// ---------------------------------------------------------------------------
// host side

int alloc_extra(gsim_handle* h)
{
    free_extra(h);
    h->x = new Extra();
    if (h->e == 0) return GSIM_OK;
    const size_t bytes = 2 * (size_t)h->e * (size_t)std::max(1, h->S);
    hipError_t e = hipMalloc((void**)&h->x->d_ctl, bytes);
    if (e != hipSuccess) return hip_check(h, e, "hipMalloc ctl");
    h->bytes_allocated += bytes;
    e = hipMemsetAsync(h->x->d_ctl, 0, bytes, h->stream);
    if (e != hipSuccess) return hip_check(h, e, "memset ctl");
    const size_t any_bytes = 2 * sizeof(uint64_t) * (size_t)h->n;
    e = hipMalloc((void**)&h->x->d_cany, any_bytes);
    if (e == hipSuccess) e = hipMemsetAsync(h->x->d_cany, 0, any_bytes, h->stream);
    if (e != hipSuccess) return hip_check(h, e, "control summary");
    h->bytes_allocated += any_bytes;
    const size_t lp_bytes = sizeof(int64_t) * (size_t)h->n * (size_t)std::max(1, h->t);
    e = hipMalloc((void**)&h->x->d_lastpub, lp_bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&h->x->d_fantopics, sizeof(uint64_t) * (size_t)h->n);
    if (e != hipSuccess) return hip_check(h, e, "hipMalloc fanout");
    h->bytes_allocated += lp_bytes + sizeof(uint64_t) * (size_t)h->n;
    e = hipMemsetAsync(h->x->d_lastpub, 0, lp_bytes, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(h->x->d_fantopics, 0, sizeof(uint64_t) * (size_t)h->n, h->stream);
    if (e != hipSuccess) return hip_check(h, e, "memset fanout");
    // the graph's uploads were queued on the handle's (non-blocking) stream: they
    // must land before the blocking reads below
    e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "graph upload");
    std::vector<uint32_t> rp((size_t)h->n + 1);
    e = stream_copy(h, rp.data(), h->d_row_ptr, sizeof(uint32_t) * rp.size(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_check(h, e, "row_ptr readback");
    uint32_t md = 0, mdall = 0;
    std::vector<uint32_t> cls[7];
    for (int64_t i = h->olo(); i < h->ohi(); ++i) {
        const uint32_t d = rp[(size_t)i + 1] - rp[(size_t)i];
        md = std::max(md, d);
        cls[d <= 16 ? 0 : d <= 32 ? 1 : d <= 64 ? 2 : d <= 256 ? 3 : d <= 1024 ? 4 : d <= 4096 ? 5 : 6].push_back((uint32_t)i);
    }
    for (int64_t i = 0; i < h->n; ++i) mdall = std::max(mdall, rp[(size_t)i + 1] - rp[(size_t)i]);
    if (!h->all_joined) {
        // lane groups pack 2-4 observers per wavefront, which runs the union of
        // their joined topics: observers with the same subscriptions side by side
        // (order within a heartbeat is free: observers are independent)
        std::vector<uint64_t> sub((size_t)h->n);
        e = stream_copy(h, sub.data(), h->d_sub, sizeof(uint64_t) * sub.size(), hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_check(h, e, "subscription readback");
        for (int c = 0; c < 2; ++c)
            std::stable_sort(cls[c].begin(), cls[c].end(), [&](uint32_t x, uint32_t y) { return sub[x] < sub[y]; });
    }
    // rows of at most 8 connections first in their class, 8 observers per wavefront
    // (a power law's many short rows idle half of a 16-lane group)
    int64_t n8 = 0;
    if (GSIM_HB_W8) {
        n8 = std::stable_partition(cls[0].begin(), cls[0].end(),
                                   [&](uint32_t x) { return rp[(size_t)x + 1] - rp[(size_t)x] <= 8; }) - cls[0].begin();
    }
    // the hub classes by row length: the shorter half of a class's range runs
    // on a block of half the threads (a 1024-thread block idles most of its
    // lanes on a row of 300), and the 1025-4096 class's first nh2048 rows take
    // 2 positions per thread (k_heartbeat_hub<1024, 2>: 4 spill registers)
    auto by_len = [&](std::vector<uint32_t>& c, uint32_t lim) {
        std::stable_sort(c.begin(), c.end(), [&](uint32_t x, uint32_t y) {
            return rp[(size_t)x + 1] - rp[(size_t)x] < rp[(size_t)y + 1] - rp[(size_t)y];
        });
        return (int64_t)std::count_if(c.begin(), c.end(), [&](uint32_t x) { return rp[(size_t)x + 1] - rp[(size_t)x] <= lim; });
    };
    h->x->nh128 = by_len(cls[3], 128);
    h->x->nh512 = by_len(cls[4], 512);
    h->x->nh2048 = by_len(cls[5], 2048);
    h->x->max_degree = md;
    h->x->n8 = n8;
    h->x->n16 = (int64_t)cls[0].size(); h->x->n32 = (int64_t)cls[1].size(); h->x->n64 = (int64_t)cls[2].size();
    h->x->nh256 = (int64_t)cls[3].size(); h->x->nh1024 = (int64_t)cls[4].size(); h->x->nh4096 = (int64_t)cls[5].size();
    h->x->nh8192 = (int64_t)cls[6].size();
    if (h->x->nh8192 > 0 && md <= kGiantRow) {
        // the giant rows' group state: one slice per block of their launches
        h->x->gscratch_blocks = std::min<int64_t>(h->x->nh8192, 64);
        const size_t gb = sizeof(typename BlockGroup<1024, kGiantRow / 1024>::Shared) * (size_t)h->x->gscratch_blocks;
        e = hipMalloc(&h->x->d_gscratch, gb);
        if (e != hipSuccess) return hip_check(h, e, "giant-row scratch");
        h->bytes_allocated += gb;
    }
    if (md > 16 || !h->all_joined || n8 > 0) {   // several classes, or an order by subscriptions: keep the lists
        std::vector<uint32_t> all;
        all.reserve((size_t)h->n);
        for (auto& c : cls) all.insert(all.end(), c.begin(), c.end());
        e = hipMalloc((void**)&h->x->d_rows, sizeof(uint32_t) * all.size());
        if (e == hipSuccess)
            e = stream_copy(h, h->x->d_rows, all.data(), sizeof(uint32_t) * all.size(), hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_check(h, e, "row classes");
        h->bytes_allocated += sizeof(uint32_t) * all.size();
    }
    h->max_degree = mdall;   // every local row (a shard's ghost rows too)
    if (h->gp.do_px) {
        const size_t pb = sizeof(uint64_t) * (size_t)h->n + 2 * (size_t)h->e + sizeof(uint32_t) * (1 + 2 * (size_t)h->e) +
                          sizeof(double) * (size_t)h->e;
        e = hipMalloc((void**)&h->x->d_pxo, sizeof(uint64_t) * (size_t)h->n);
        if (e == hipSuccess) e = hipMalloc((void**)&h->x->d_pxm, (size_t)h->e);
        if (e == hipSuccess) e = hipMalloc((void**)&h->x->d_nopx, (size_t)h->e);
        if (e == hipSuccess) e = hipMalloc((void**)&h->x->d_pxc, sizeof(uint32_t) * (1 + 2 * (size_t)h->e));
        if (e == hipSuccess) e = hipMalloc((void**)&h->x->d_pxs, sizeof(double) * (size_t)h->e);
        if (e == hipSuccess) e = hipMalloc((void**)&h->x->d_pxl_n, 2 * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemsetAsync(h->x->d_pxl_n, 0, 2 * sizeof(uint32_t), h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(h->x->d_pxo, 0, sizeof(uint64_t) * (size_t)h->n, h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(h->x->d_pxm, 0, (size_t)h->e, h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(h->x->d_nopx, 0, (size_t)h->e, h->stream);
        if (e != hipSuccess) return hip_check(h, e, "peer exchange state");
        h->bytes_allocated += pb;
    }
    return GSIM_OK;
}

void free_extra(gsim_handle* h)
{
    if (!h->x) return;
    if (h->x->d_ctl) (void)hipFree(h->x->d_ctl);
    if (h->x->d_cany) (void)hipFree(h->x->d_cany);
    if (h->x->d_rows) (void)hipFree(h->x->d_rows);
    if (h->x->d_gscratch) (void)hipFree(h->x->d_gscratch);
    if (h->x->d_lastpub) (void)hipFree(h->x->d_lastpub);
    if (h->x->d_fantopics) (void)hipFree(h->x->d_fantopics);
    if (h->x->d_pxo) (void)hipFree(h->x->d_pxo);
    if (h->x->d_pxm) (void)hipFree(h->x->d_pxm);
    if (h->x->d_nopx) (void)hipFree(h->x->d_nopx);
    if (h->x->d_pxc) (void)hipFree(h->x->d_pxc);
    if (h->x->d_pxs) (void)hipFree(h->x->d_pxs);
    if (h->x->d_pxl) (void)hipFree(h->x->d_pxl);
    if (h->x->d_pxl_tick) (void)hipFree(h->x->d_pxl_tick);
    if (h->x->d_pxl_n) (void)hipFree(h->x->d_pxl_n);
    delete h->x;
    h->x = nullptr;
}

// The inbox was written through the ABI: any topic of any receiver may hold
// entries, so the next control pass reads every plane once.
int extra_field_written(gsim_handle* h, int32_t f)
{
    if (f != GSIM_F_CTL || !h->x || !h->x->d_cany) return GSIM_OK;
    return hip_check(h, hipMemsetAsync(h->x->d_cany, 0xFF, 2 * sizeof(uint64_t) * (size_t)h->n, h->stream),
                     "control summary");
}

uint8_t* extra_ctl(gsim_handle* h) { return h->x ? h->x->d_ctl : nullptr; }
uint8_t** extra_ctl_slot(gsim_handle* h)
{
    static uint8_t* none = nullptr;
    return h->x ? &h->x->d_ctl : &none;
}
uint64_t* extra_cany(gsim_handle* h) { return h->x ? h->x->d_cany : nullptr; }

bool extra_field_ref(gsim_handle* h, int32_t f, gsim::FieldRef* r)
{
    if (f == GSIM_F_CTL && h->x && h->x->d_ctl) {
        *r = {h->x->d_ctl, 2 * (size_t)h->e * (size_t)std::max(1, h->t), FK_TEDGE, 1, 2};
        return true;
    }
    if (f == GSIM_F_LASTPUB && h->x && h->x->d_lastpub) {
        *r = {h->x->d_lastpub, sizeof(int64_t) * (size_t)h->n * (size_t)std::max(1, h->t)};
        return true;
    }
    if (f == GSIM_F_FANOUT_TOPICS && h->x && h->x->d_fantopics) {
        *r = {h->x->d_fantopics, sizeof(uint64_t) * (size_t)h->n};
        return true;
    }
    return false;
}

static HbArgs make_hb_args(gsim_handle* h, uint64_t tick, int64_t now, int parity_in)
{
    HbArgs a{};
    a.N = h->n; a.E = h->e; a.T = h->t;
    a.row_ptr = h->d_row_ptr; a.col = h->d_col; a.rev = h->d_rev; a.sub = h->d_sub; a.smask = h->d_smask;
    a.outbound = h->d_outbound; a.direct = h->d_direct; a.estate = h->d_estate; a.score = h->d_score; a.tp = h->d_tp;
    a.tflags = h->d_tflags; a.mflags = h->d_mflags; a.rstate = h->d_rstate; a.backoff = h->d_backoff; a.meshd = h->d_meshd; a.fail = h->d_fail; a.bp = h->d_bp;
    a.graft = h->d_graft; a.mtime = h->d_mtime; a.mcnt = h->d_mcnt;
    // a Graft before the last refresh's time would read as older than it is
    // (lazy_mtime): a clock that runs backwards stores meshTime again
    if (h->mt_lazy && now < h->mt_R) (void)materialize_mtime(h, true);
    a.mt_lazy = h->mt_lazy ? 1 : 0;
    a.mt_R = h->mt_R;
    const size_t TE = (size_t)h->e * (size_t)std::max(1, h->S);
    a.ctl_in = h->x->d_ctl + (size_t)(parity_in & 1) * TE;
    a.ctl_out = h->x->d_ctl + (size_t)((parity_in + 1) & 1) * TE;
    a.cany_in = h->x->d_cany + (size_t)(parity_in & 1) * (size_t)h->n;
    a.cany_out = h->x->d_cany + (size_t)((parity_in + 1) & 1) * (size_t)h->n;
    a.tick = tick; a.now = now; a.seed = h->x->seed;
    a.D = h->gp.d; a.Dlo = h->gp.dlo; a.Dhi = h->gp.dhi; a.Dscore = h->gp.dscore; a.Dout = h->gp.dout;
    a.opp_peers = h->gp.opportunistic_graft_peers; a.opp_ticks = h->gp.opportunistic_graft_ticks;
    a.prune_backoff = h->gp.prune_backoff_ns; a.graft_flood = h->gp.graft_flood_threshold_ns;
    a.unsub_backoff = h->gp.unsubscribe_backoff_ns;
    a.opp_threshold = h->th.opportunistic_graft_threshold;
    GossipView gv{};
    a.gossip = deliver_gossip_view(h, &gv);
    a.lastput = gv.lastput; a.gsel = gv.gsel; a.gstate = gv.gstate; a.mmask = a.gossip ? gv.mmask : nullptr;
    a.gossip_thr = h->th.gossip_threshold; a.gossip_factor = h->gp.gossip_factor;
    a.dlazy = h->gp.dlazy; a.hist_gossip = h->gp.history_gossip;
    a.first = h->d_first; a.invalid = h->d_invalid; a.p5 = h->d_p5; a.p6 = h->d_p6;
#ifndef GSIM_HB_SUB_GATHER
    a.sub_all = h->all_joined && !h->sub_dynamic ? 1 : 0;
#endif
#ifndef GSIM_HB_INV_GATHER
    a.inv_live = h->d_inv_live ? h->d_inv_live + (h->inv_par & 1) : nullptr;
#endif
    a.topic_cap = h->pp.topic_score_cap; a.w5 = h->pp.app_specific_weight; a.w6 = h->pp.ip_colocation_factor_weight;
    a.bp_thr = h->pp.behaviour_penalty_threshold; a.w7 = h->pp.behaviour_penalty_weight;
    a.lastpub = h->x->d_lastpub; a.fan_topics = h->x->d_fantopics;
    a.pub_thr = h->th.publish_threshold; a.fanout_ttl = h->gp.fanout_ttl_ns;
    a.gid = h->sh ? h->sh->d_gid : nullptr;
    // (push: no shard reads a ghost row's router state)
    if (ShardCtx* sh = h->sh; sh && sh->d_rdel && !sh->push) {
        a.rdel = sh->d_rdel;
        a.rdel_n = sh->d_rdel_n;
        a.rdel_cap = sh->rdel_cap;
        a.xq = sh->d_xq;
        a.sr.K = sh->K;
        a.sr.self = sh->k;
        for (int q = 0; q <= sh->K; ++q) a.sr.lo[q] = sh->lpeer[(size_t)q];
    }
    a.olo = (uint32_t)h->olo();
    a.ohi = (uint32_t)h->ohi();
    const bool push = h->sh && h->sh->push;
    a.mlo = push ? 0u : a.olo;
    a.mhi = push ? (uint32_t)h->n : a.ohi;
    a.do_px = h->x->d_pxo ? 1 : 0;
    a.prune_peers = h->gp.prune_peers;
    a.accept_px = h->th.accept_px_threshold;
    a.pxo = h->x->d_pxo; a.pxm = h->x->d_pxm; a.nopx = h->x->d_nopx; a.pxs = h->x->d_pxs;
    a.pxl = h->x->d_pxl; a.pxl_tick = h->x->d_pxl_tick; a.pxl_n = h->x->d_pxl_n; a.pxl_cap = h->x->pxl_cap;
    if (ShardCtx* sh = h->sh; sh && sh->d_pxout && a.do_px) {
        a.pxout = sh->d_pxout; a.pxcnt = sh->d_pxcnt; a.pxcap = sh->pxcap; a.pxK = sh->K;
        a.xre = sh->d_xre; a.pshard = sh->d_pshard;
    }
    a.tr = h->trace;
    return a;
}

static int grid_rows(int64_t n)
{
    int64_t g = (n + 3) / 4;
    return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 65536);
}

static int check_degree(gsim_handle* h)
{
    if (h->x->max_degree > (uint32_t)kGiantRow) {
        h->err = "heartbeat kernels support rows of at most 8192 connections in this build";
        return GSIM_ERANGE;
    }
    return GSIM_OK;
}

uint64_t gsim_get_seed(const gsim_handle* h) { return h->x ? h->x->seed : 0; }

int launch_fanout_publish(gsim_handle* h, const gsim_msg* d_pub, int32_t count, int64_t g, int64_t now)
{
    if (h->gp.flood_publish || count <= 0 || !h->x || !h->x->d_lastpub) return GSIM_OK;
    HbArgs a = make_hb_args(h, (uint64_t)g, now, 0);
    hipLaunchKernelGGL(k_fanout_publish, dim3((count + 3) / 4), dim3(256), 0, h->stream, a, d_pub, count);
    if (h->x->nh256 + h->x->nh1024)
        hipLaunchKernelGGL((k_fanout_publish_hub<1024, 1>), dim3(count), dim3(1024), 0, h->stream, a, d_pub, count, 64u);
    if (h->x->nh4096)
        hipLaunchKernelGGL((k_fanout_publish_hub<1024, 4>), dim3(count), dim3(1024), 0, h->stream, a, d_pub, count,
                           1024u);
    if (h->x->nh8192)
        hipLaunchKernelGGL((k_fanout_publish_hub_g<1024, kGiantRow / 1024>),
                           dim3((uint32_t)std::min<int64_t>(count, h->x->gscratch_blocks)), dim3(1024), 0, h->stream, a,
                           d_pub, count, 4096u, h->x->d_gscratch);
    return hip_check(h, hipGetLastError(), "k_fanout_publish");
}

extern "C" {

int gsim_set_seed(gsim_handle* h, uint64_t seed)
{
    if (!h || !h->x) return GSIM_EINVAL;
    h->x->seed = seed;
    return GSIM_OK;
}

int gsim_heartbeat(gsim_handle* h, uint64_t tick, int64_t now)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->e == 0 || !h->x) { h->err = "no graph loaded"; return GSIM_ESTATE; }
    int rc = check_degree(h);
    if (!rc && !h->in_step) rc = deliver_check_errors(h);   // (gsim_step reads them once per call)
    if (rc) return rc;
    rc = deliver_flush(h);
    if (!rc) rc = deliver_heartbeat_begin(h, tick);   // IHAVE marks of this heartbeat are pending
    if (rc) return rc;
    // heartbeat output goes to the parity-0 inbox, read by control round 0
    HbArgs a = make_hb_args(h, tick, now, 1);
    ProfScope ps(h, GSIM_K_HEARTBEAT);
    // observers in lane groups sized to their rows: 4 per wavefront for rows
    // of <= 16 connections, 2 for <= 32, 1 otherwise (observers are
    // independent within a heartbeat, so the classes run one after the other)
    const Extra* x = h->x;
    const int64_t nown = h->ohi() - h->olo();
    if (x->n16 == nown && !x->d_rows) {   // one class: the owned rows in order
        hipLaunchKernelGGL(k_heartbeat<16>, dim3(grid_rows((nown + 3) / 4)), dim3(256), 0, h->stream, a, nullptr, nown,
                           h->olo());
    } else if (x->n32 == nown && !x->d_rows) {
        hipLaunchKernelGGL(k_heartbeat<32>, dim3(grid_rows((nown + 1) / 2)), dim3(256), 0, h->stream, a, nullptr, nown,
                           h->olo());
    } else if (x->n64 == nown && !x->d_rows) {
        hipLaunchKernelGGL(k_heartbeat<64>, dim3(grid_rows(nown)), dim3(256), 0, h->stream, a, nullptr, nown, h->olo());
    } else {
        const uint32_t* r = x->d_rows;
        if (x->n8) hipLaunchKernelGGL(k_heartbeat<8>, dim3(grid_rows((x->n8 + 7) / 8)), dim3(256), 0, h->stream,
                                      a, r, x->n8, (int64_t)0);
        if (x->n16 > x->n8)
            hipLaunchKernelGGL(k_heartbeat<16>, dim3(grid_rows((x->n16 - x->n8 + 3) / 4)), dim3(256), 0, h->stream,
                               a, r + x->n8, x->n16 - x->n8, (int64_t)0);
        if (x->n32) hipLaunchKernelGGL(k_heartbeat<32>, dim3(grid_rows((x->n32 + 1) / 2)), dim3(256), 0, h->stream,
                                       a, r + x->n16, x->n32, (int64_t)0);
        if (x->n64) hipLaunchKernelGGL(k_heartbeat<64>, dim3(grid_rows(x->n64)), dim3(256), 0, h->stream,
                                       a, r + x->n16 + x->n32, x->n64, (int64_t)0);
        // hubs: one block per observer
        const uint32_t* rh = r + x->n16 + x->n32 + x->n64;
        // one block per class row: (threads, row positions per thread) by class (kHub*)
        auto hub = [&](auto kern, int bt, int64_t off, int64_t n) {
            if (n > 0)
                hipLaunchKernelGGL(kern, dim3((uint32_t)std::min<int64_t>(n, 65536)), dim3(bt), 0, h->stream, a, rh + off, n);
        };
        hub(k_heartbeat_hub<kHubB[0], kHubVv[0]>, kHubB[0], 0, x->nh128);
        hub(k_heartbeat_hub<kHubB[1], kHubVv[1]>, kHubB[1], x->nh128, x->nh256 - x->nh128);
        hub(k_heartbeat_hub<kHubB[2], kHubVv[2]>, kHubB[2], x->nh256, x->nh512);
        hub(k_heartbeat_hub<kHubB[3], kHubVv[3]>, kHubB[3], x->nh256 + x->nh512, x->nh1024 - x->nh512);
        hub(k_heartbeat_hub<kHubB[4], kHubVv[4]>, kHubB[4], x->nh256 + x->nh1024, x->nh2048);
        hub(k_heartbeat_hub<kHubB[5], kHubVv[5]>, kHubB[5], x->nh256 + x->nh1024 + x->nh2048, x->nh4096 - x->nh2048);
        if (x->nh8192)   // 8 row positions per thread, group state in global scratch
            hipLaunchKernelGGL((k_heartbeat_hub_g<1024, kGiantRow / 1024>), dim3((uint32_t)x->gscratch_blocks), dim3(1024),
                               0, h->stream, a, rh + x->nh256 + x->nh1024 + x->nh4096, x->nh8192, x->d_gscratch);
    }
    hipLaunchKernelGGL(k_fanout_heartbeat, dim3(grid_rows(nown)), dim3(256), 0, h->stream, a);
    const uint32_t* rh = x->d_rows + x->n16 + x->n32 + x->n64;
    if (x->nh256)
        hipLaunchKernelGGL((k_fanout_heartbeat_hub<256, 1>), dim3((uint32_t)std::min<int64_t>(x->nh256, 65536)),
                           dim3(256), 0, h->stream, a, rh, x->nh256);
    if (x->nh1024)
        hipLaunchKernelGGL((k_fanout_heartbeat_hub<1024, 1>), dim3((uint32_t)std::min<int64_t>(x->nh1024, 65536)),
                           dim3(1024), 0, h->stream, a, rh + x->nh256, x->nh1024);
    if (x->nh4096)
        hipLaunchKernelGGL((k_fanout_heartbeat_hub<1024, 4>), dim3((uint32_t)std::min<int64_t>(x->nh4096, 65536)),
                           dim3(1024), 0, h->stream, a, rh + x->nh256 + x->nh1024, x->nh4096);
    if (x->nh8192)
        hipLaunchKernelGGL((k_fanout_heartbeat_hub_g<1024, kGiantRow / 1024>), dim3((uint32_t)x->gscratch_blocks),
                           dim3(1024), 0, h->stream, a, rh + x->nh256 + x->nh1024 + x->nh4096, x->nh8192, x->d_gscratch);
    if (a.do_px)    // sendGraftPrune's makePrune with PX, live scores after every topic
        launch_px_emit(h, a, 1, (uint32_t)tick, (uint32_t)P_PX);
    return hip_check(h, hipGetLastError(), "k_heartbeat");
}

}  // extern "C"

int handle_control(gsim_handle* h, int32_t round, int64_t now)
{
    HbArgs a = make_hb_args(h, 0, now, round & 1);
    ProfScope ps(h, GSIM_K_CONTROL);
    hipLaunchKernelGGL(k_handle_control, dim3(grid_rows(h->ohi() - h->olo())), dim3(256), 0, h->stream, a);
    if (a.do_px) {  // handleGraft's PRUNE replies with PX (snapshot scores)
        const uint32_t kt = (uint32_t)((uint64_t)now ^ ((uint64_t)now >> 32));
        launch_px_emit(h, a, 0, kt, (uint32_t)P_PX_GRAFT);
    }
    return hip_check(h, hipGetLastError(), "k_handle_control");
}

extern "C" {

int gsim_handle_control(gsim_handle* h, int32_t round, int64_t now)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->e == 0 || !h->x) { h->err = "no graph loaded"; return GSIM_ESTATE; }
    int rc = check_degree(h);
    if (rc) return rc;
    return handle_control(h, round, now);
}


int gsim_read_snapshot(gsim_handle* h, int64_t obs_lo, int64_t obs_hi, gsim_peer_score_snapshot* peers,
                       gsim_topic_score_snapshot* topics)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->e == 0 || !h->x) { h->err = "no graph loaded"; return GSIM_ESTATE; }
    if (obs_lo < 0 || obs_hi > h->n || obs_lo > obs_hi || (!peers && obs_hi > obs_lo)) {
        h->err = "observer range out of bounds";
        return GSIM_EINVAL;
    }
    int rc = deliver_flush(h);                    // first deliveries of the last round are credited
    if (!rc && h->p6_dirty) rc = launch_ip_colocation(h);
    if (rc) return rc;
    uint32_t rp[2];
    hipError_t e = stream_copy(h, rp, h->d_row_ptr + obs_lo, sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = stream_copy(h, rp + 1, h->d_row_ptr + obs_hi, sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_check(h, e, "row bounds");
    const int64_t ne = (int64_t)rp[1] - rp[0], T = std::max(1, h->t);
    if (ne == 0) return GSIM_OK;
    gsim_peer_score_snapshot* dp = nullptr;
    gsim_topic_score_snapshot* dt = nullptr;
    e = hipMalloc((void**)&dp, sizeof(*dp) * (size_t)ne);
    if (e == hipSuccess) e = hipMalloc((void**)&dt, sizeof(*dt) * (size_t)(ne * T));
    if (e == hipSuccess) {
        HbArgs a = make_hb_args(h, 0, h->mt_R, 0);   // (no clock read; the last refresh's keeps meshTime lazy)
        hipLaunchKernelGGL(k_snapshot, dim3((uint32_t)std::min<int64_t>((ne + 255) / 256, 16384)), dim3(256), 0,
                           h->stream, a, (int64_t)rp[0], (int64_t)rp[1], dp, dt);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(peers, dp, sizeof(*dp) * (size_t)ne, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && topics)
        e = hipMemcpyAsync(topics, dt, sizeof(*dt) * (size_t)(ne * T), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (dp) (void)hipFree(dp);
    if (dt) (void)hipFree(dt);
    return hip_check(h, e, "gsim_read_snapshot");
}

}  // extern "C"

// AddPeer / RemovePeer at both ends of connections given as device edges:
// edges[2q + d] = the edge of direction d of connection q (n2 = 2 * count).
static int apply_connections(gsim_handle* h, const uint32_t* d_edges, int32_t n2, int32_t up, int64_t now)
{
    const int grid = (n2 + 255) / 256;
    HbArgs a = make_hb_args(h, 0, now, 0);   // ctl_in/ctl_out cover both inbox planes
    ChurnArgs c{};
    c.edges = d_edges; c.n2 = n2; c.up = up ? 1 : 0; c.retain = h->pp.retain_score_ns;
    c.estate = h->d_estate; c.rstate = h->d_rstate; c.pen = h->d_pen; c.expire = h->d_expire;
    c.first = h->d_first; c.invalid = h->d_invalid;
    c.skip_unjoined = h->unjoined_zero ? 1 : 0;
    c.p6row = h->d_p6row;
    hipLaunchKernelGGL(k_churn_apply, dim3(grid), dim3(256), 0, h->stream, a, c);
    const hipError_t e = hipGetLastError();   // stream-ordered: the next call's copy into the scratch follows this kernel
    if (e != hipSuccess) return hip_check(h, e, "k_churn_apply");
    const int rcg = gater_connections(h, d_edges, n2, up, now);   // the peer gater's AddPeer / RemovePeer
    if (rcg) return rcg;
    h->p6_dirty = true;          // the tracked set (and so the IP sets) changed
    if (!up) h->maybe_retained = true;
    h->score_version++;          // connected / tracked bits feed the delivery state (churn only clears mesh bits: the masks stay a superset)
    return GSIM_OK;
}

extern "C" {

int gsim_set_connections(gsim_handle* h, const uint32_t* pairs, int32_t count, int32_t up, int64_t now)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->e == 0 || !h->x) { h->err = "no graph loaded"; return GSIM_ESTATE; }
    if (count < 0 || (count > 0 && !pairs)) { h->err = "bad connection list"; return GSIM_EINVAL; }
    if (count == 0) return GSIM_OK;
    // the pairs' edges, found (and checked) before anything changes: a pair
    // that is not a connection, or a connection listed twice (it would be
    // handled by two threads at once), fails the call
    const int32_t n2 = 2 * count;
    hipError_t e = hipSuccess;
    const int64_t need = 2 * (int64_t)n2 + 2;   // pairs, edges, bad[2]
    if (h->churn_cap < need) {   // grow-only scratch: no allocation (and no hipFree sync) per call
        if (h->d_churn) { (void)hipFree(h->d_churn); h->d_churn = nullptr; h->churn_cap = 0; }
        e = hipMalloc((void**)&h->d_churn, sizeof(uint32_t) * (size_t)need);
        if (e == hipSuccess) h->churn_cap = need;
    }
    if (e == hipSuccess && !h->d_churn_mark) {
        const size_t words = ((size_t)h->e + 31) / 32;
        e = hipMalloc((void**)&h->d_churn_mark, sizeof(uint32_t) * words);
        if (e == hipSuccess) e = hipMemsetAsync(h->d_churn_mark, 0, sizeof(uint32_t) * words, h->stream);
    }
    uint32_t* d_pairs = h->d_churn;
    uint32_t* d_edges = d_pairs + n2;
    uint32_t* d_bad = d_edges + n2;
    if (e == hipSuccess) e = hipMemcpyAsync(d_pairs, pairs, sizeof(uint32_t) * (size_t)n2, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d_bad, 0xFF, 2 * sizeof(uint32_t), h->stream);
    uint32_t bad[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
    const int grid = (n2 + 255) / 256;
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_churn_find, dim3(grid), dim3(256), 0, h->stream, (const uint32_t*)h->d_row_ptr,
                           (const uint32_t*)h->d_col, h->n, (const uint32_t*)d_pairs, n2, d_edges, d_bad,
                           h->d_churn_mark);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_churn_unmark, dim3(grid), dim3(256), 0, h->stream, (const uint32_t*)d_pairs,
                           (const uint32_t*)d_edges, n2, h->d_churn_mark);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(bad, d_bad, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);   // a bad list fails the call before any change
    if (e != hipSuccess) return hip_check(h, e, "gsim_set_connections");
    if (bad[0] != 0xFFFFFFFFu) {
        h->err = "pair " + std::to_string(bad[0]) + " is not a connection";
        return GSIM_EINVAL;
    }
    if (bad[1] != 0xFFFFFFFFu) {
        h->err = "pair " + std::to_string(bad[1]) + ": the connection is listed twice";
        return GSIM_EINVAL;
    }
    int rc = deliver_flush(h);              // pending first deliveries precede the removal
    // the P3b test reads meshMessageDeliveries: k_churn_apply applies the pending
    // increments of the records it removes (GSIM_CHURN_MCNT), else a pass over all
    if (!rc && !GSIM_CHURN_MCNT) rc = materialize_mcnt(h);
    // RemovePeer scores the peer live (score.go:611-644): P6 over the tracked
    // set as it is now (an up batch since the last derivation changed it)
    if (!rc && !up && h->p6_dirty) rc = launch_ip_colocation(h);
    if (rc) return rc;
    ProfScope ps(h, GSIM_K_CHURN);
    return apply_connections(h, d_edges, n2, up, now);
}

int gsim_set_subscriptions(gsim_handle* h, const uint32_t* pairs, int32_t count, int32_t join, uint64_t tick,
                           int64_t now)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->e == 0 || !h->x) { h->err = "no graph loaded"; return GSIM_ESTATE; }
    if (count < 0 || (count > 0 && !pairs)) { h->err = "bad subscription list"; return GSIM_EINVAL; }
    if (count == 0) return GSIM_OK;
    const int32_t T = std::max(1, h->t);
    std::vector<uint64_t> need;
    for (int32_t q = 0; q < count; ++q) {
        if ((int64_t)pairs[2 * q] >= h->n || (int32_t)pairs[2 * q + 1] >= T) {
            h->err = "subscription pair out of range";
            return GSIM_EINVAL;
        }
        // a joining peer's router state for the topic lives in its topic slot
        if (join && !h->smask.empty() && !((h->smask[pairs[2 * q]] >> pairs[2 * q + 1]) & 1ull)) {
            if (need.empty()) need.assign((size_t)h->n, 0);
            need[pairs[2 * q]] |= 1ull << pairs[2 * q + 1];
        }
    }
    int rc = deliver_flush(h);
    if (!rc) rc = materialize_mcnt(h);       // stats_prune reads meshMessageDeliveries
    if (!rc && !need.empty()) rc = ensure_slots(h, need.data());
    if (rc) return rc;
    ProfScope ps(h, GSIM_K_CHURN);
    const int64_t words = 2 * (int64_t)count + 2;   // pairs, then one u64 (Leave's PX room)
    if (h->churn_cap < words) {
        if (h->d_churn) { (void)hipFree(h->d_churn); h->d_churn = nullptr; h->churn_cap = 0; }
        const hipError_t e = hipMalloc((void**)&h->d_churn, sizeof(uint32_t) * (size_t)words);
        if (e != hipSuccess) return hip_check(h, e, "gsim_set_subscriptions");
        h->churn_cap = words;
    }
    hipError_t e = hipMemcpyAsync(h->d_churn, pairs, sizeof(uint32_t) * 2 * (size_t)count, hipMemcpyHostToDevice,
                                  h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_set_subscriptions");
    if (!join && h->x->d_pxo) {
        // room for Leave's PX lists: PrunePeers entries per connection of a leaving peer
        unsigned long long* d_sum = reinterpret_cast<unsigned long long*>(h->d_churn + 2 * (size_t)count);
        e = hipMemsetAsync(d_sum, 0, sizeof(unsigned long long), h->stream);
        if (e == hipSuccess)
            hipLaunchKernelGGL(k_pair_degrees, dim3(1), dim3(256), 0, h->stream, (const uint32_t*)h->d_row_ptr,
                               (const uint32_t*)h->d_churn, count, d_sum);
        unsigned long long sum = 0;
        uint32_t cur[2] = {0, 0};
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(&sum, d_sum, sizeof(sum), hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(cur, h->x->d_pxl_n, sizeof(cur), hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return hip_check(h, e, "Leave PX room");
        const int64_t need = (int64_t)cur[0] + (int64_t)sum * std::max(0, h->gp.prune_peers);
        if (need > h->x->pxl_cap) {
            const int64_t cap = need + need / 2 + 1024;
            uint64_t* nl = nullptr;
            uint32_t* nt = nullptr;
            e = hipMalloc((void**)&nl, sizeof(uint64_t) * (size_t)cap);
            if (e == hipSuccess) e = hipMalloc((void**)&nt, sizeof(uint32_t) * (size_t)cap);
            if (e == hipSuccess && cur[0] && h->x->d_pxl) {
                e = hipMemcpyAsync(nl, h->x->d_pxl, sizeof(uint64_t) * cur[0], hipMemcpyDeviceToDevice, h->stream);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(nt, h->x->d_pxl_tick, sizeof(uint32_t) * cur[0], hipMemcpyDeviceToDevice, h->stream);
                if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
            }
            if (e != hipSuccess) {
                if (nl) (void)hipFree(nl);
                if (nt) (void)hipFree(nt);
                return hip_check(h, e, "Leave PX lists");
            }
            if (h->x->d_pxl) (void)hipFree(h->x->d_pxl);
            if (h->x->d_pxl_tick) (void)hipFree(h->x->d_pxl_tick);
            h->x->d_pxl = nl;
            h->x->d_pxl_tick = nt;
            h->bytes_allocated += 12 * (size_t)(cap - h->x->pxl_cap);
            h->x->pxl_cap = cap;
        }
    }
    HbArgs a = make_hb_args(h, tick, now, 1);   // ctl_out: the heartbeat's inbox (control round 0)
    hipLaunchKernelGGL(k_subscribe, dim3(1), dim3(64), 0, h->stream, a, h->d_sub, (const uint32_t*)h->d_churn, count,
                       join ? 1 : 0);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "k_subscribe");
    h->mesh_version++;            // router mesh / fanout bits changed: delivery masks rebuild
    h->score_version++;
    if (!join) {
        h->unjoined_zero = false; // a peer that left keeps records of the topic
        h->all_joined = false;
        h->sub_dynamic = true;    // receivers may hold copies of topics they left
    }
    return GSIM_OK;
}

int gsim_px_connect(gsim_handle* h, int64_t now, uint32_t* pairs, int64_t cap, int64_t* n_connected)
{
    if (!h || !n_connected) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    *n_connected = 0;
    if (h->e == 0 || !h->x) { h->err = "no graph loaded"; return GSIM_ESTATE; }
    if (!h->x->d_pxm) return GSIM_OK;                     // WithPeerExchange is off
    int rc0 = px_leave_import(h, nullptr);                 // Leave's PRUNEs: the pruned peers' PX handling
    if (rc0) return rc0;
    uint32_t* pxc = h->x->d_pxc;
    hipError_t e = hipMemsetAsync(pxc, 0, sizeof(uint32_t), h->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_px_collect, dim3((uint32_t)std::min<int64_t>((h->e + 255) / 256, 16384)), dim3(256), 0,
                           h->stream, (const uint32_t*)h->d_owner, (const uint32_t*)h->d_col,
                           (const uint32_t*)h->d_rev, (const uint8_t*)h->d_rstate, h->x->d_pxm, h->e, pxc);
        e = hipGetLastError();
    }
    uint32_t n = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&n, pxc, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_px_connect");
    *n_connected = n;
    if (n == 0) return GSIM_OK;
    if (pairs && cap > 0) {
        // (dialer, peer) of every connection, sorted (4n <= 2E: after the edge list)
        hipLaunchKernelGGL(k_px_pairs, dim3((n + 255) / 256), dim3(256), 0, h->stream, (const uint32_t*)pxc, n,
                           (const uint32_t*)h->d_owner, (const uint32_t*)h->d_col, pxc + 1 + 2 * (size_t)n);
        std::vector<uint32_t> pv(2 * (size_t)n);
        e = hipGetLastError();
        if (e == hipSuccess)
            e = hipMemcpyAsync(pv.data(), pxc + 1 + 2 * (size_t)n, sizeof(uint32_t) * pv.size(), hipMemcpyDeviceToHost,
                               h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return hip_check(h, e, "gsim_px_connect pairs");
        std::vector<std::pair<uint32_t, uint32_t>> pr((size_t)n);
        for (size_t q = 0; q < n; ++q) pr[q] = {pv[2 * q], pv[2 * q + 1]};
        std::sort(pr.begin(), pr.end());
        for (size_t q = 0; q < n && (int64_t)q < cap; ++q) { pairs[2 * q] = pr[q].first; pairs[2 * q + 1] = pr[q].second; }
    }
    int rc = deliver_flush(h);                    // as gsim_set_connections
    if (!rc && !GSIM_CHURN_MCNT) rc = materialize_mcnt(h);
    if (rc) return rc;
    ProfScope ps(h, GSIM_K_CHURN);
    hipLaunchKernelGGL(k_px_outbound, dim3((n + 255) / 256), dim3(256), 0, h->stream, (const uint32_t*)pxc, n,
                       h->d_outbound);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_check(h, e, "k_px_outbound");
    return apply_connections(h, pxc + 1, (int32_t)(2 * n), 1, now);
}

}  // extern "C"

#ifdef GSIM_DIAG_HB
// the diagnostic counters (not part of gsim.h): read, then reset
extern "C" int gsim_diag_hb_counts(gsim_handle* h, uint64_t* out4)
{
    if (!h || !out4) return GSIM_EINVAL;
    if (hipStreamSynchronize(h->stream) != hipSuccess) return GSIM_EDEVICE;
    unsigned long long z[4] = {0, 0, 0, 0};
    if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_hb_diag), sizeof(z)) != hipSuccess) return GSIM_EDEVICE;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_hb_diag), z, sizeof(z)) != hipSuccess) return GSIM_EDEVICE;
    return GSIM_OK;
}
#endif
