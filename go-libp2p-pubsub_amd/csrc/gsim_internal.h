// gsim_internal.h — engine handle and kernel argument blocks (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "gsim.h"

// Every host synchronisation the library makes is counted (gsim_host_sync_count,
// include/gsim.h): stream synchronisations and blocking copies.  The per-tick
// count is the host round trips a caller's tick pays (bench.py reports it).
#include <atomic>
namespace gsim {
extern std::atomic<unsigned long long> g_host_syncs;
inline hipError_t counted_stream_sync(hipStream_t s)
{
    g_host_syncs.fetch_add(1, std::memory_order_relaxed);
    return (hipStreamSynchronize)(s);
}
inline hipError_t counted_memcpy(void* dst, const void* src, size_t n, hipMemcpyKind k)
{
    g_host_syncs.fetch_add(1, std::memory_order_relaxed);
    return (hipMemcpy)(dst, src, n, k);
}
}  // namespace gsim
#define hipStreamSynchronize(s) ::gsim::counted_stream_sync(s)
#define hipMemcpy(d, s, n, k) ::gsim::counted_memcpy(d, s, n, k)

namespace gsim {

constexpr int GSIM_MAX_TOPICS = 64;   // subscriptions are a u64 bitmask
constexpr int kEvents = 512;

struct ScoreArgs {
    int64_t E;
    int32_t T;
    const gsim_topic_score_params* tp;
    double dtz, bp_decay, topic_cap, w5, w6, bp_thr, w7;
    const uint32_t* owner;     // owner[r]: the neighbour a record is about (§2)
    const double* p5;
    double *first, *meshd, *fail, *invalid;
    uint8_t* mcnt;             // pending meshMessageDeliveries increments (see apply_incs)
    int64_t *graft, *mtime;
    uint8_t* tflags;           // score bits only (inMesh, active)
    uint8_t* mflags;           // router mesh bits, edge order (fill/census)
    uint8_t* rstate;           // router connected bit, edge order (fill)
    const uint32_t* rev;
    double* bp;
    uint8_t* pen;              // pending P7 penalty counts, added after the decay
    uint8_t* estate;
    int64_t* expire;
    const double* p6;
    double* score;
    int64_t now;
    int32_t mt_lazy;           // lazy meshTime (lazy_mtime): in-mesh records were not stored at the last refresh
    int64_t mt_R;              // ... whose time this is
    int32_t* purged;
    const uint64_t* sub;       // announced topics per peer (fill: records only where both endpoints joined)
    const int32_t* gate;       // non-null: run only if *gate != 0 (a retention purge happened)
    const uint32_t* col;       // col[r]: the observer of record r (record order)
    const uint64_t* smask;     // topic slots of each row owner (nullptr: dense, slot = topic)
    int32_t S;                 // planes per topic array
    int32_t skip_unjoined;     // records of topics the observer did not join are zero: skip them
    // sharded network: only records whose observer is owned
    // ([olo, ohi)) are this shard's; the owned rows are local edges [e_lo, e_hi),
    // global edge index geid_base + (e - e_lo) of E_glob
    int32_t sharded;
    uint32_t olo, ohi;
    int64_t e_lo, e_hi, geid_base, E_glob;
    uint8_t* p6row;            // [N] a purge marks its observer's row for the next P6 pass
    // invalidMessageDeliveries is zero in every record while *inv_live is 0
    // (Handle::d_inv_live): the pass reads no invalid plane then, and a
    // refresh sets *inv_next when a record still holds a non-zero value
    const uint32_t* inv_live;
    uint32_t* inv_next;
};

struct ColocArgs {
    int64_t E;
    const uint32_t *row_ptr, *col, *rev, *owner, *ip_ptr, *ip_ids;
    const uint8_t* ip_white;
    const uint8_t* estate;
    double* p6;
    int32_t thr;
    const int32_t* gate;       // non-null: run only if *gate != 0 (a retention purge happened)
    int32_t sharded;           // only owned observers ([olo, ohi)) get P6
    uint32_t olo, ohi;
    uint32_t hub_min;          // rows longer than this are the hub kernel's (k_ip_colocation_hub)
    uint8_t* rowflag;          // non-null: only rows flagged here are re-derived (and their flags cleared)
};

// meshMessageDeliveries increments from message delivery are kept as a
// per-record u8 count between score passes (the delivery kernel then touches
// one byte per copy instead of read-modify-writing an f64): applying them is
// the exact sequence of markDuplicate/markFirst updates x -> min(x + 1, cap)
// (score.go:935-941, 975-980), performed before anything reads the counter.
__device__ __forceinline__ double apply_incs(double x, uint32_t n, double cap)
{
    for (uint32_t k = 0; k < n; ++k) {
        x = x + 1.0;
        if (x > cap) { x = cap; break; }   // further increments keep the cap
    }
    return x;
}

// Exact Go int64 division (truncation toward zero) of meshTime by a positive
// TimeInMeshQuantum (score.go:287): an fp64 quotient estimate corrected by the
// exact integer remainder.  Cheaper in VALU and registers than the generic
// 64-bit division expansion; the result is identical for every input.
__device__ __forceinline__ int64_t div_trunc_pos(int64_t n, int64_t d)
{
    const bool neg = n < 0;
    const uint64_t un = neg ? (uint64_t)0 - (uint64_t)n : (uint64_t)n;
    const uint64_t ud = (uint64_t)d;
    uint64_t q = (uint64_t)((double)un / (double)ud);
    // the estimate is within a few units of the true quotient; fix it exactly
    while (q * ud > un) --q;
    while (un - q * ud >= ud) ++q;
    return neg ? -(int64_t)q : (int64_t)q;
}

__device__ __forceinline__ int64_t go_div(int64_t n, int64_t d)
{
    return d > 0 ? div_trunc_pos(n, d) : n / d;
}

// A kernel's first argument re-read from the kernarg segment behind an opaque
// pointer: loads of its fields stay where they are used (scalar loads, K$
// hits) instead of being hoisted out of the loops, where dozens of live
// pointers overflow the SGPRs and spill to VGPR lanes (a v_readlane per use).
// Only valid in a kernel whose FIRST parameter is the A passed, unmodified:
// a helper reached from another kernel, or handed a modified copy, would read
// the wrong memory silently.  Debug builds (GSIM_DEBUG_KERNARG, `make debug`)
// trap when the re-read struct's leading 16 bytes differ from the argument's.
template <class A>
__device__ __forceinline__ const A& kernarg0(const A& arg)
{
    using CP = const __attribute__((address_space(4))) A*;
    CP p = (CP)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
#ifdef GSIM_DEBUG_KERNARG
    static_assert(sizeof(A) >= 16, "kernarg0 check reads 16 bytes");
    const uint64_t* x = (const uint64_t*)&arg;
    const __attribute__((address_space(4))) uint64_t* y = (const __attribute__((address_space(4))) uint64_t*)p;
    if (x[0] != y[0] || x[1] != y[1]) __builtin_trap();
#else
    (void)arg;
#endif
    return *(const A*)p;
}

// meshTime of an in-mesh record of a connected, tracked peer in a scored
// topic — the records refreshScores rewrites (score.go:550-556) — once the
// engine stopped storing it (lazy meshTime): the last refresh
// at R left R - graftTime there, and a Graft since then (graftTime >= R)
// stored 0 itself.  Stored values stay authoritative until the first refresh
// (lazy = 0) and for a graft time after R (Graft's 0, or a refresh that met a
// graft time in the future and stored its negative meshTime).
__device__ __forceinline__ int64_t lazy_mtime(int32_t lazy, int64_t R, int64_t graft, int64_t stored)
{
    return lazy && graft <= R ? R - graft : stored;
}

// Topic slots.  Every per-(topic, edge index) array — score
// records in record order, router state in edge order — holds S planes, not
// T: the plane of topic t at index x is the rank of t in the slot mask of x's
// row owner (owner[x]: the neighbour for a record, the observer for router
// state).  A row owner's mask covers every topic it ever joined or published
// to, and a record (i about j, t) can only be non-zero if j has t (j
// forwarded, was grafted for or sent control on t), so nothing outside the
// masks is ever stored.  All-joined networks keep S = T and smask == nullptr:
// the plane of t is t, as a dense [T][E] layout.
__device__ __forceinline__ uint64_t smask_of(const uint64_t* smask, uint32_t owner)
{
    return smask ? smask[owner] : ~0ull;
}
__device__ __forceinline__ bool slot_has(uint64_t m, int32_t t) { return (m >> t) & 1ull; }
__device__ __forceinline__ int64_t slot_idx(uint64_t m, int32_t t, int64_t E, int64_t x)
{
    return (int64_t)__popcll(m & ((1ull << t) - 1ull)) * E + x;
}
// topic of the p-th plane of a row owner with mask m (p < popcount(m))
__device__ __forceinline__ int32_t slot_topic(uint64_t m, int32_t p)
{
    for (int32_t k = 0; k < p; ++k) m &= m - 1;
    return m ? __builtin_ctzll(m) : -1;
}

// Topic parameters are read-only for a kernel's lifetime.  Reading them
// through the constant address space (4) lets the compiler use scalar
// s_load (scalar cache, lgkmcnt) instead of vector loads that it must order
// against the kernel's stores with s_waitcnt vmcnt(0) — which serializes every
// memory round trip of the hot loops.
typedef const __attribute__((address_space(4))) gsim_topic_score_params* ctp_t;
__device__ __forceinline__ ctp_t const_tp(const gsim_topic_score_params* p)
{
    return (ctp_t)(p);
}

// How a field's ABI (edge-order) view maps onto device memory.
enum FieldKind : int {
    FK_RAW = 0,      // same layout
    FK_RECORD,       // per edge, record order: view[e] = dev[rev[e]]
    FK_TRECORD,      // topic slots, record order: view[t][e] = dev[slot][rev[e]]
    FK_TEDGE,        // topic slots, edge order: view[par][t][e] = dev[par][slot][e]
    FK_TFLAGS,       // view = score bits (record order) | router mesh bit (edge order)
    FK_ESTATE,       // record order + router connected mirror (edge order)
    FK_SEEN,         // first-seen rounds: the high words of the 64-bit seen-set cells (read-only)
};

struct FieldRef {
    void* ptr;
    size_t bytes;      // of the ABI view
    int kind = FK_RAW;
    int elem = 1;      // element size in bytes
    int npar = 1;      // FK_TEDGE: [npar] sets of topic planes
};

struct Deliver;   // message ring, seen-set and round lists (deliver.hip)

// A shard of a graph-sharded network (shard.hip): which local
// peers / edges the handle owns and the device side of the halo exchange.
// A handle without one owns every peer (sh == nullptr).
// A shard's view of the peer ranges (kernel argument): local ids
// [lo[s], lo[s+1]) are shard s's peers; self = this shard.
struct ShardRanges {
    int64_t lo[GSIM_MAX_SHARDS + 1];
    int32_t K, self;
};

// One source shard's part of a tick's received holder bits (k_holder_import):
// n slots' ids at in_off, then n x nw words over its owned peers; bit b of
// word w of a slot is global peer pbase + 64 w + b.
struct HSrc {
    int64_t in_off, pbase, toff;
    int32_t n, nw;
};

// One source shard's part of a round's received copy bits (k_xbits_deliver):
// its n active slots' ids at in_off, then n x xw words; bit b of slot k is a
// copy on record gbase + b (the ghost block of the source's peers).
struct XSrc {
    int64_t in_off;    // first entry of the source's part (slot ids, then words)
    int64_t gbase;     // first record of its ghost block
    int64_t toff;      // first wave task (64 words of one slot each)
    int32_t n, xw;     // slots, words per slot
};

struct ShardCtx {
    int32_t k = 0, K = 1;
    int64_t own_lo = 0, own_hi = 0;        // owned local peers
    int64_t own_e_lo = 0, own_e_hi = 0;    // local edges of the owned rows
    int64_t N_global = 0, E_global = 0;
    int64_t geid_base = 0;                 // global edge index of own_e_lo
    std::vector<int64_t> bounds;           // [K+1] global peer ranges
    std::vector<int64_t> lpeer;            // [K+1] local ids of each shard's peers
    std::vector<int64_t> gbase, gcnt;      // [K] ghost rows of shard s's peers (local edges)
    std::vector<int64_t> xoff;             // [K+1] cross-out lists, concatenated (d_xgather)
    uint32_t* d_gid = nullptr;             // [n] global id of each local peer
    uint32_t* d_g2l = nullptr;             // [N_global] local id of a global peer (0xFFFFFFFF: not local)
    uint32_t* d_ymap = nullptr;            // [e] ghost-row edge: the owner shard's owned-row edge index
    uint32_t* d_xgather = nullptr;         // [n_cross] cross-out lists (local edge indices)
    uint32_t* d_xpos = nullptr;            // [e] its inverse: an owned-row cross edge's index in them (~0: none)
    uint8_t* d_pgate = nullptr;            // [e] ghost-row edge: the sender's score of the receiver >= publishThreshold
    int64_t send_edges = 0, send_max = 0;  // edges into owned peers, longest such run of a row
    uint32_t* d_xq = nullptr;              // [e] owned-row cross edge: its position in the cross-out list to its shard
    uint64_t* d_rdel = nullptr;            // control-round router changes of cross edges (k_handle_control)
    uint32_t* d_rdel_n = nullptr;
    int64_t rdel_cap = 0;
    uint64_t* d_rdel_in = nullptr;         // ... every other shard's
    int64_t rdel_in_cap = 0;
    uint32_t* d_sptr = nullptr;            // [n+1] CSR of each row's edges into owned peers (the copies this shard delivers)
    uint32_t* d_sedge = nullptr;           // their local edge indices, in row order
    std::vector<uint8_t> xto;              // [K] the owned peers have connections into shard q's
    // frontier exchange (gsim_group_msgs_init)
    uint64_t* d_fout = nullptr;            // owned forwarders of the round (k_frontier_export)
    uint32_t* d_fcnt = nullptr;
    int64_t fcap = 0;
    int64_t fpend = 0;                     // push: entries accumulated since the last flush (one per tick)
    uint64_t* d_fin = nullptr;             // every other shard's forwarders
    int64_t fin_cap = 0;
    // push: the holders of a tick as bits (a ghost's cell is read by IHAVE
    // only, at tick granularity): [2][ring][how] by the tick's parity, over
    // the owned peers' global words; the slots touched [2][ring/32]
    uint64_t* d_hbits = nullptr;
    uint32_t* d_hslots = nullptr;
    int64_t how = 0;                       // owned global words
    int32_t hring = 0;
    uint64_t* d_hsend = nullptr;           // [ring * (1 + how)] the tick's slots, then their words
    uint32_t* d_hn = nullptr;              // [1] its slots
    HSrc* d_hsrc = nullptr;                // [K] the received parts
    HSrc* h_hsrc = nullptr;                // pinned staging of it
    // control exchange
    uint64_t* d_cout = nullptr;            // [K][ccap] outbound control entries: edge | topic << 32 | bits << 40
    uint32_t* d_ccnt = nullptr;            // [K]
    int64_t ccap = 0;
    uint64_t* d_cin = nullptr;             // inbound control entries
    int64_t cin_cap = 0;
    // router state of cross edges (mesh / fanout masks, connected | direct | publish gate)
    uint64_t *d_rmesh_out = nullptr, *d_rfan_out = nullptr;   // [n_cross]
    uint8_t* d_rflag_out = nullptr;
    uint64_t *d_rmesh_in = nullptr, *d_rfan_in = nullptr;     // [e] (ghost-row positions)
    uint8_t* d_rflag_in = nullptr;
    // gossip marks of cross edges
    uint64_t* d_gout = nullptr;            // [n_cross] topic mask of gsel
    uint8_t* d_gsout = nullptr;            // [n_cross] gstate
    uint64_t* d_gin = nullptr;             // [e] (ghost-row positions)
    uint8_t* d_gsin = nullptr;             // [e]
    uint32_t* h_counts = nullptr;          // pinned scratch for count readbacks
    // copy push: a round's copies from owned senders to ghost
    // receivers go to the receivers' shards as bits, per (destination, slot)
    // one bit per cross edge into the destination, in its cross-out order
    bool push = true;
    std::vector<int64_t> rbase;            // [K] first local edge of this shard's ghost block at shard d
    uint32_t* d_xre = nullptr;             // [e] owned-row cross edge: the edge's index at the receiver's shard (PX)
    uint8_t* d_pshard = nullptr;           // [n] shard of each local peer
    std::vector<int64_t> xwo;              // [K+1] word offset of each destination's segment in a slot's row
    int64_t* d_xwo = nullptr;              // ... on the device
    int64_t xbw = 0;                       // words per slot row (xwo[K])
    uint32_t* d_xwq = nullptr;             // [e] owned-row cross edge: its bit in a slot's row (64 xwo[d] + position)
    uint64_t* d_xbits = nullptr;           // [ring][xbw] the round's copies to ghost receivers (k_send_tm<PUSH>)
    int32_t xring = 0;                     // slots d_xbits holds
    uint64_t* d_xsend = nullptr;           // [K][xsend_cap] per destination: the active slots, then their segments
    int64_t xsend_cap = 0;
    uint64_t* d_xrecv = nullptr;           // the same from every other shard
    int64_t xrecv_cap = 0;
    uint32_t* d_xn = nullptr;              // [1] active slots of the round (k_xbits_gather)
    uint32_t* h_xcnt = nullptr;            // pinned: its readback
    XSrc* d_xsrc = nullptr;                // [K] the received parts (k_xbits_deliver)
    XSrc* h_xsrc = nullptr;                // pinned staging of it
    // peer exchange to ghosts (k_px_emit's remote path, gsim_group_px_connect)
    uint64_t* d_pxout = nullptr;           // [K][pxcap] PX list entries per destination shard
    uint32_t* d_pxcnt = nullptr;           // [K + 1] their counts, overflow
    int64_t pxcap = 0;
    uint64_t* d_pxin = nullptr;            // entries from the other shards / the job's attempts / its connections
    int64_t pxin_cap = 0;
};

// Seen-set cells [ring][N] (deliver.hip): unseen; committed (hi = first-seen
// round, lo = first sender); or claimed in round g (hi = kClaim | parity of g
// << 30 | claiming edge, lo = sender | credit flags).
constexpr uint64_t kUnseen64 = ~0ull;
constexpr uint32_t kClaim = 0x80000000u;
constexpr uint32_t kEdgeMask = 0x3FFFFFFFu;       // claim edge bits (E < 2^30 - 1)
constexpr uint32_t kCreditFirst = 0x80000000u;     // lo-word flag: winner's record gets P2
constexpr uint32_t kCreditMesh = 0x40000000u;      // lo-word flag: ... and P3 (negative window)
constexpr uint32_t kPeerMask = 0x3FFFFFFFu;

// The seen-set (a21): one 64-bit cell (encoding above) per
// (ring slot, peer that can see the slot's message).  A ring shared by every
// topic (slot = id % ring) and a topic every peer holds: a cell per peer,
// cbase[m] + p.  Per-topic sub-rings (gsim_msg_config.topic_slots) of a topic
// only some peers hold — its members, the peers with a slot for it (§2) —
// keep one cell per member, in peer order: cbase[m] + the member's index,
// found from a word of the topic's member bitmap and the members before it.
struct Cells {
    uint64_t* cell = nullptr;
    const uint64_t* cbase = nullptr;   // [ring] first cell of each slot
    const uint64_t* mbits = nullptr;   // [T][nw] member bits of each topic (sparse topics)
    const uint32_t* mpre = nullptr;    // [T][nw] members in the topic's earlier words
    int64_t nw = 0;                    // words per topic, ceil(N / 64)
    int64_t n = 0;                     // peers
    uint64_t sparse = 0;               // topics whose slots hold member-compacted cells
    // (no sparse topic: every slot holds a cell per peer at m * n + p, no table read)
    // word w of topic t: its member bits and the cell offset of its first member
    __device__ __forceinline__ void word(int32_t t, int64_t w, uint64_t& bits, int64_t& pre) const
    {
        if ((sparse >> t) & 1ull) {
            const int64_t i = (int64_t)t * nw + w;
            bits = mbits[i];
            pre = mpre[i];
        } else {
            bits = ~0ull;
            pre = w * 64;
        }
    }
    // cell index of peer p in slot m (topic t) whose cells start at base; -1: p has none
    __device__ __forceinline__ int64_t at(int64_t base, int32_t t, uint32_t p) const
    {
        if (!((sparse >> t) & 1ull)) return base + p;
        uint64_t b;
        int64_t pre;
        word(t, (int64_t)(p >> 6), b, pre);
        const uint64_t bit = 1ull << (p & 63);
        if (!(b & bit)) return -1;
        return base + pre + __popcll(b & (bit - 1));
    }
    __device__ __forceinline__ int64_t idx(uint32_t m, int32_t t, uint32_t p) const
    {
        if (!sparse) return (int64_t)m * n + p;
        return at((int64_t)cbase[m], t, p);
    }
    __device__ __forceinline__ uint64_t get(uint32_t m, int32_t t, uint32_t p) const
    {
        const int64_t i = idx(m, t, p);
        return i < 0 ? kUnseen64 : cell[i];
    }
};

// Trace capture (gsim_trace_config, include/gsim.h): the events of the
// routers [lo, hi) are appended to a device buffer.  A message copy is
// recorded unclassified (kTraceCopy, msg_id = round << 32 | slot) and resolved
// into DELIVER / REJECT / DUPLICATE against the seen-set cell when read.
constexpr uint8_t kTraceCopy = 0xFF;
struct TraceRef {
    gsim_trace_event* ev = nullptr;
    uint32_t* n = nullptr;
    int64_t cap = 0;
    uint32_t lo = 0, hi = 0;          // traced routers this engine owns (a shard: local ids)
    uint32_t xlo = 0, xhi = 0;        // ... and its ghosts in the traced range (a shard; else = lo, hi)
    // host bookkeeping: events [0, resolved) of the buffer were resolved by an
    // earlier gsim_trace_read and kept for a later one (their ids are wire ids:
    // resolving them again would index the slot arrays with a message id)
    uint32_t resolved = 0;
    __device__ __forceinline__ bool on(uint32_t p) const { return ev != nullptr && p >= lo && p < hi; }
    // a traced router that may be another shard's ghost here: events only
    // this shard knows of (the RecvRPC of a copy it pushes, the SendRPC of an
    // IWANT answer or the RecvRPC of an IWANT request whose other end is a ghost)
    __device__ __forceinline__ bool on_any(uint32_t p) const { return ev != nullptr && p >= xlo && p < xhi; }
    __device__ __forceinline__ void push(int64_t ts, uint64_t mid, uint32_t peer, uint32_t other, int32_t topic,
                                         uint8_t type, uint8_t reason) const
    {
        const uint32_t k = atomicAdd(n, 1u);
        if ((int64_t)k >= cap) return;                 // counted: gsim_trace_read reports the overflow
        gsim_trace_event x;
        x.timestamp_ns = ts; x.msg_id = mid; x.peer = peer; x.other = other; x.topic = topic;
        x.type = type; x.reason = reason; x._pad = 0;
        ev[k] = x;
    }
};

struct Gater;   // the peer gater's state (gater.hip)

// The peer gater's device state as the delivery kernels see it (gater.hip;
// act == nullptr: the gater is off).
struct GaterRef {
    const uint8_t* act = nullptr;        // [N] the receiver's gate may throttle this round
    const uint32_t* gq = nullptr;        // [E] record order: the receiver's IP group of the sender (edge order)
    const double *del = nullptr, *dup = nullptr, *ign = nullptr, *rej = nullptr;
    unsigned long long* a_del = nullptr; // the round's events
    uint32_t *a_dup = nullptr, *a_ign = nullptr, *a_rej = nullptr, *a_val = nullptr, *a_thr = nullptr;
    uint8_t* a_last = nullptr;
    const unsigned long long* tw = nullptr;   // [T] delivery weights (2^-16 units)
    double dw = 0, iw = 0, rw = 0;
    uint64_t seed = 0;
    unsigned long long* n_thr = nullptr;
    const uint8_t* direct = nullptr;     // [E] edge order: gs.direct (AcceptFrom: AcceptAll)
    uint32_t* prom = nullptr;            // [P][E] IWANT promises (ThrottlePeer forgets the peer's)
    int32_t P = 0;
    const uint32_t* gid = nullptr;       // a shard: global id of each local peer (the draw's key)
};

}  // namespace gsim

struct gsim_handle {
    int device = 0;
    bool validate = true;
    hipStream_t stream = nullptr;
    hipEvent_t ev[gsim::kEvents] = {};
    std::string err;

    gsim_peer_score_params pp{};
    std::vector<gsim_topic_score_params> tp;
    gsim_thresholds th{};
    gsim_gossipsub_params gp{};
    int32_t t = 0;

    int64_t n = 0, e = 0;
    // topic slots (smask_of above): S planes per topic array; d_smask is null
    // while every peer holds every topic (S = T)
    int32_t S = 0;
    std::vector<uint64_t> smask;   // host copy of the slot masks (empty: dense)
    uint64_t* d_smask = nullptr;
    uint32_t n_ips = 0;
    uint32_t max_degree = 0;   // longest CSR row (set when the graph is loaded)
    size_t bytes_allocated = 0;
    bool has_white = false;
    bool p6_dirty = true;
    // only the rows flagged in d_p6row changed (churn, retention purges): the
    // P6 pass re-derives those; false: every row (graph, IPs, whitelist, writes)
    bool p6_rows_only = false;
    // some IP is held by two local peers (gsim_set_ips / load): otherwise every
    // peersInIP is 1 and P6 is 0 everywhere (launch_ip_colocation)
    bool ip_shared = false;
    bool maybe_retained = false;
    // Every record of a topic its observer did not join is zero (true after
    // gsim_load_graph and gsim_fill_synthetic, false after any state write
    // through the ABI).  Subscriptions are fixed and nothing on the path
    // touches such a record (deliveries, GRAFT/PRUNE and gossip reach joined
    // topics only), so they stay zero and the score pass may skip them.
    bool unjoined_zero = false;
    bool all_joined = false;     // every peer announced every topic (nothing to skip)
    bool sub_dynamic = false;    // a Leave happened: receivers check the copy's topic (gsim_set_subscriptions)
    std::vector<int64_t> topic_subs;   // [T] local peers that joined each topic (k_send_tm's block shares)
    bool tm_uniform = false;  // k_send_tm blocks the same for every topic (gsim_set_kernel_variant(h, 6, 1))
    int64_t tm_budget = 0;    // k_send_tm blocks in all (0: ranges x T, launch_send_tm_tb)
    int ihave_w = 0;          // k_ihave lane group width (gsim_set_kernel_variant(h, 3, w)); 0 = by row lengths
    bool xb_generic = false;  // k_xbits_deliver: listed_copy only, never the batched path (variant 8, 1)
    bool flist_off = false;   // never the list-driven send k_send_list (gsim_set_kernel_variant(h, 9, 1))
    bool in_step = false;     // inside gsim_step: the error flags are read once per call, not per heartbeat

    // device: parameters and scratch flags
    gsim_topic_score_params* d_tp = nullptr;
    int32_t* d_flags = nullptr;
    // [2] invalidMessageDeliveries flags: d_inv_live[inv_par] != 0 unless every
    // record's counter is zero.  Written by the copies that raise a counter
    // (deliver.hip inv_mark) and set by any state write through the ABI; a
    // refresh reads it, writes the exact flag of the decayed state into the
    // other word and flips inv_par (engine.hip launch_refresh_scores)
    uint32_t* d_inv_live = nullptr;
    int inv_par = 0;

    // device: graph
    uint32_t *d_row_ptr = nullptr, *d_col = nullptr, *d_rev = nullptr, *d_owner = nullptr;
    uint64_t* d_sub = nullptr;
    uint8_t* d_outbound = nullptr;
    uint8_t* d_direct = nullptr;       // [E] edge order: col[e] is in the observer's gs.direct set
    uint32_t *d_ip_ptr = nullptr, *d_ip_ids = nullptr;
    uint8_t* d_ip_white = nullptr;
    double* d_p5 = nullptr;

    // Score state is stored in RECORD order: the record of
    // observer i about neighbour j sits at index r = rev[e_ij], i.e. at the
    // position of i in j's row, so a message j forwards updates its receivers'
    // records with coalesced accesses along j's row.  rev is an involution,
    // so the ABI's edge-order view is a gather through rev both ways.
    // device: topicStats [T][E], record order
    double *d_first = nullptr, *d_meshd = nullptr, *d_fail = nullptr, *d_invalid = nullptr;
    uint8_t* d_mcnt = nullptr;        // pending meshd increments (apply_incs)
    bool mcnt_dirty = false;
    int64_t *d_graft = nullptr, *d_mtime = nullptr;
    bool mt_lazy = false;             // lazy meshTime since the refresh at mt_R (lazy_mtime)
    int64_t mt_R = 0;
    uint8_t* d_tflags = nullptr;      // GSIM_TF_IN_MESH | GSIM_TF_ACTIVE
    // device: router state [T][E] / [E], edge (observer) order
    uint8_t* d_mflags = nullptr;      // GSIM_TF_MESH: gs.mesh[topic] membership
    int64_t* d_backoff = nullptr;
    uint8_t* d_rstate = nullptr;      // GSIM_ES_CONNECTED as the router sees it

    // device: peerStats [E], record order
    double* d_bp = nullptr;
    uint8_t* d_estate = nullptr;
    int64_t* d_expire = nullptr;
    double* d_p6 = nullptr;
    uint8_t* d_p6row = nullptr;       // [N] the observer's tracked set changed since its last P6
    uint32_t* d_churn = nullptr;      // gsim_set_connections scratch: [cap] pairs, [cap] edges, [2] bad / twice
    int64_t churn_cap = 0;            // u32 words allocated at d_churn
    uint32_t* d_churn_mark = nullptr; // [E/32] connections listed in the current call (zero between calls)
    double* d_score = nullptr;
    uint8_t* d_pen = nullptr;         // pending broken-promise penalties (applyIwantPenalties), record order
    uint8_t* d_dstate = nullptr;      // delivery state per edge, derived (GSIM_DS_*)
    uint64_t score_version = 1, acc_version = 0;
    uint64_t mesh_version = 1;   // router mesh / direct flags changed (delivery rebuilds its mesh masks)

    // per-kernel-class device timing (gsim_profile); events are pooled
    struct ProfMark { int32_t cls; uint32_t a, b; };
    bool prof_on = false;
    bool prof_lost = false;
    std::vector<hipEvent_t> prof_pool;
    size_t prof_used = 0;
    std::vector<ProfMark> prof_marks;

    // heartbeat state lives in heartbeat.hip, message propagation in deliver.hip
    struct Extra* x = nullptr;
    gsim::Deliver* dl = nullptr;
    gsim::ShardCtx* sh = nullptr;   // graph-sharded network: this handle is one shard (shard.hip)
    struct gsim::Gater* gt = nullptr;   // peer gater (gater.hip), nullptr: off
    gsim::TraceRef trace;           // gsim_trace_config (trace.hip)

    // owned peers / observer rows (all of them unless sharded)
    int64_t olo() const { return sh ? sh->own_lo : 0; }
    int64_t ohi() const { return sh ? sh->own_hi : n; }
};

int hip_check(gsim_handle* h, hipError_t e, const char* what);
// The handle's stream is non-blocking: nothing orders it with the null
// stream's hipMemcpy / hipMemset.  Copies and fills go through the stream
// (a copy waits for it: the host buffer may be released on return).
inline hipError_t stream_copy(gsim_handle* h, void* dst, const void* src, size_t bytes, hipMemcpyKind kind)
{
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, h->stream);
    return e == hipSuccess ? hipStreamSynchronize(h->stream) : e;
}
inline hipError_t stream_fill(gsim_handle* h, void* dst, int value, size_t bytes)
{
    return hipMemsetAsync(dst, value, bytes, h->stream);
}
bool field_ref(gsim_handle* h, int32_t f, gsim::FieldRef* r);
int trace_config_local(gsim_handle* h, uint32_t peer_lo, uint32_t peer_hi, uint32_t xlo, uint32_t xhi, int64_t cap);
int launch_ip_colocation(gsim_handle* h, const int32_t* gate = nullptr);
int launch_refresh_scores(gsim_handle* h, int64_t now);
int launch_compute_scores(gsim_handle* h);
int refresh_accept(gsim_handle* h);   // recompute d_dstate if the snapshot changed
int materialize_mcnt(gsim_handle* h); // apply pending meshd increments everywhere
// store every lazy meshTime (lazy_mtime) — before meshTime is read out — and
// with leave, end lazy mode: before state is written through the ABI, topic
// parameters change or the clock runs backwards
int materialize_mtime(gsim_handle* h, bool leave);
// grow the topic slot masks to cover need[N] (a host array; the topic arrays are re-laid out)
int ensure_slots(gsim_handle* h, const uint64_t* need);
uint8_t** extra_ctl_slot(gsim_handle* h);        // heartbeat.hip: the [2][S][E] control inbox
uint8_t** deliver_gsel_slot(gsim_handle* h);     // deliver.hip: the [S][E] emitGossip choices
int slots_changed(gsim_handle* h);               // deliver.hip: member spaces follow the masks
// Publish's fanout branch for a batch already on the device (heartbeat.hip)
int launch_fanout_publish(gsim_handle* h, const gsim_msg* d_pub, int32_t count, int64_t g, int64_t now);

// Delivery state byte per edge index e: what one forwarded
// copy over e needs besides the topic planes.
enum : uint8_t {
    GSIM_DS_CONNECTED = 0x01,   // router: the sender (row owner) is connected to col[e]
    GSIM_DS_ACCEPT = 0x02,      // record e: the receiver accepts RPCs from the sender (AcceptFrom)
    GSIM_DS_TRACKED = 0x04,     // record e: the receiver keeps peerStats for the sender
    GSIM_DS_DIRECT = 0x08,      // router: col[e] is one of the sender's direct peers (always sent to)
};

// Brackets the launches of one kernel class with pooled HIP events on the
// engine stream while profiling is enabled (gsim_profile).
struct ProfScope {
    gsim_handle* h;
    int32_t cls;
    int32_t a;
    ProfScope(gsim_handle* hh, int32_t c);
    ~ProfScope();
};

// implemented in heartbeat.hip
int alloc_extra(gsim_handle* h);
void free_extra(gsim_handle* h);
bool extra_field_ref(gsim_handle* h, int32_t f, gsim::FieldRef* r);
int extra_field_written(gsim_handle* h, int32_t f);

// implemented in deliver.hip
void free_deliver(gsim_handle* h);
bool deliver_field_ref(gsim_handle* h, int32_t f, gsim::FieldRef* r);
int deliver_flush(gsim_handle* h);                  // commit the last round's claims (if any)

// What the heartbeat's emitGossip needs from the message state.
struct GossipView {
    const int32_t* lastput;   // [T][N] tick of the newest mcache.Put
    uint8_t* gsel;            // [T][E] sender edge order: emitGossip chose col[e] this heartbeat
    uint8_t* gstate;          // [E] edge order: owner's snapshot score of col >= gossipThreshold
    uint64_t* mmask;          // [T][N] delivery's mesh masks (rows <= 64), kept current by the router kernels
};
bool deliver_gossip_view(gsim_handle* h, GossipView* v);   // false before gsim_msgs_init
// What the wire encoder reads of the message state (wire.hip)
struct WireView {
    gsim::Cells cells;         // the seen-set
    const uint32_t *mtopic, *morigin;
    const uint8_t* minv;
    const uint64_t* mid;       // [ring] gsim_msg ids
    const int32_t* slot_last;  // [ring] last round with a new claim or the publication
    const uint8_t* gsel;       // [T][E] emitGossip's targets (sender edge order)
    int32_t ring, rounds;
    int64_t ihave_tick;        // heartbeat whose gossip is pending, -1 none
};
bool deliver_wire_view(gsim_handle* h, WireView* v);     // false before gsim_msgs_init
// What the wire encoder needs of peer exchange (heartbeat.hip): the PX
// observers' live scores, the selection seed, Leave's kept PX lists; false
// when WithPeerExchange is off
struct WirePx {
    const double* pxs;
    uint64_t seed;
    const uint64_t* pxl;
    const uint32_t* pxl_tick;
    uint32_t n_pxl;
};
bool deliver_wire_px(gsim_handle* h, WirePx* w);
int deliver_promise_check(gsim_handle* h, int64_t now);    // broken promises -> pending P7
int deliver_heartbeat_begin(gsim_handle* h, uint64_t tick); // fresh IHAVE marks
uint64_t gsim_get_seed(const gsim_handle* h);              // heartbeat.hip
int deliver_read_seen(gsim_handle* h, void* dst);
int deliver_check_errors(gsim_handle* h);             // queue overflow / early slot reuse of the last tick
int handle_control(gsim_handle* h, int32_t round, int64_t now);   // heartbeat.hip: k_handle_control
// heartbeat.hip, a shard's peer exchange (gsim_group_px_connect): remote PX lists in,
// its connection attempts out (global asker | peer << 32), gs.outbound of the connections
bool px_enabled(const gsim_handle* h);
int px_import(gsim_handle* h, const uint64_t* d_in, int64_t n);
// The heartbeat's row classes (heartbeat.hip): the owned observers by row
// length, rows[0, n16) of at most 16 connections, then <= 32, <= 64, then the
// hub rows (nhub, more than 64).  rows == nullptr: one class holds every owned
// observer, in order from olo.
struct RowClasses {
    const uint32_t* rows;
    int64_t n16, n32, n64, nhub;
};
void row_classes(gsim_handle* h, RowClasses* rc);
int px_leave_import(gsim_handle* h, const uint32_t* g2l);
int px_asks(gsim_handle* h, uint64_t* d_out, uint32_t* d_cnt, int64_t cap);
int px_mark_outbound(gsim_handle* h, const uint64_t* d_pairs, int64_t n);
// trace.hip: resolve the recorded message copies (seen-set cells, slot tables)
struct TraceView {
    gsim::Cells cells;
    const uint32_t* mtopic;
    const uint8_t* minv;
    const uint64_t* mid;
    int32_t ring, rounds;
    const uint8_t* mlat;        // validation latencies (nullptr: all 0)
    int64_t t0, hb;             // round times (RoundArgs)
    const int64_t* roff;
};
bool deliver_trace_view(gsim_handle* h, TraceView* v);
int64_t deliver_last_round_time(gsim_handle* h);   // time of the last round run (INT64_MAX: none yet)
void trace_release(gsim_handle* h);   // trace.hip
// round stages (deliver.hip; gsim_round runs them in order, a sharded group
// exchanges between them, shard.hip)
int deliver_round_prepare(gsim_handle* h, int64_t round);
int deliver_round_send(gsim_handle* h, int64_t round);
int deliver_round_queue(gsim_handle* h, int64_t round, const uint64_t* q, const uint32_t* d_n, int64_t cap);
int deliver_round_post(gsim_handle* h, int64_t round);
int deliver_round_control(gsim_handle* h, int64_t round);
int deliver_round_ihave(gsim_handle* h, int64_t round);
int deliver_round_validate(gsim_handle* h, int64_t round);
void deliver_round_end(gsim_handle* h, int64_t round);
int32_t* deliver_slot_last(gsim_handle* h);           // [ring]
int deliver_frontier_export(gsim_handle* h, int64_t round, uint64_t* out, uint32_t* d_cnt, int64_t cap,
                            bool append = false);
int deliver_xbits_apply(gsim_handle* h, int64_t round, const uint64_t* in, const gsim::XSrc* d_src, int K, int64_t ntask);
int deliver_holder_accum(gsim_handle* h, int64_t round);
void deliver_mcnt_applied(gsim_handle* h);
int deliver_holder_gather(gsim_handle* h, int parity);
int deliver_holder_import(gsim_handle* h, int64_t round, const uint64_t* in, const gsim::HSrc* d_src, int K,
                          int64_t ntask, int64_t fr);
int deliver_frontier_import(gsim_handle* h, int64_t round, const uint64_t* in, int64_t n);
void deliver_blocks_changed(gsim_handle* h);          // gsim_set_kernel_variant(h, 6, v)
// gater.hip: the peer gater (gsim_set_peer_gater)
gsim::GaterRef gater_ref(gsim_handle* h);
int gater_round_begin(gsim_handle* h, int64_t now);        // AcceptFrom preamble of the round
void gater_round_sent(gsim_handle* h, int64_t round);      // the round's events await its commit
int gater_fold(gsim_handle* h, int64_t round, int64_t now); // after the commit of `round`
int gater_decay(gsim_handle* h, int64_t now);               // decayStats (at the refresh)
int gater_connections(gsim_handle* h, const uint32_t* d_edges, int32_t n2, int32_t up, int64_t now);
void free_gater(gsim_handle* h);
bool deliver_latency_on(gsim_handle* h);                    // deliver.hip: a vdelay > 0 message was published
// heartbeat.hip: the control inbox ([2][T][E] by round parity) and its per-receiver summary ([2][N])
uint8_t* extra_ctl(gsim_handle* h);
uint64_t* extra_cany(gsim_handle* h);
