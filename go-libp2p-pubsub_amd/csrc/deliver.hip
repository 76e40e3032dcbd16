// deliver.hip — message propagation rounds for the whole network.
//
// Reference path (one message copy arriving at one router):
//   AcceptFrom graylist            gossipsub.go:598-609
//   pushMsg seen check / markSeen  pubsub.go:1118-1162, 987-995
//   DeliverMessage / DuplicateMessage / RejectMessage
//                                  score.go:693-827 -> markFirst/Duplicate/
//                                  InvalidMessageDelivery score.go:901-981
//   Publish forwarding to mesh     gossipsub.go:975-1045
//
// Bulk-synchronous restatement.  The seen-set is the only
// message state: one 64-bit cell per (slot, peer),
//   committed   hi = first-seen round,                lo = sender of the first copy
//   claimed     hi = 0x80000000 | parity << 30 | edge, lo = sender | credit flags
//   unseen      all ones
// so the forwarding frontier of round g-1 is every cell whose first-seen
// round is g-1 (committed, or claimed in round g-1) and no per-copy list is
// ever materialized.  One kernel per round:
//   k_send  one wave per 64 consecutive peers, for every slot that had new
//           claims in round g-1 (a coalesced load of the wave's cells):
//           (1) commit: a cell claimed in round g-1 becomes committed and its
//               winner's record gets markFirstMessageDelivery's P2 credit;
//           (2) forward: each frontier sender walks its row with a lane group
//               and, for every mesh target, evaluates AcceptFrom, loads the
//               receiver's cell and applies the score tracer to the
//               RECEIVER's record of the sender — in record order (DESIGN.md
//               §2) that record sits at the sender's own edge index, so the
//               counter traffic is coalesced along the sender's row.  A copy
//               to a cell first seen in an earlier round is a duplicate
//               (validated = that round); a copy to an unseen cell or one
//               claimed this round claims it with a 64-bit atomicMin: the
//               lowest edge — the lowest sender — wins.  Every same-round
//               copy, first or duplicate, has validated = now and so the same
//               counter update; only the P2 credit needs the winner, and it
//               is applied when the claim is committed.
//   k_commit commits the claims of the last round before anything else reads
//           the state (end of a tick, field reads), and k_reset_slots those of
//           a slot being reused.
// Counter updates are plain read-modify-writes: meshMessageDeliveries and
// invalidMessageDeliveries of a record (receiver i, sender j) are only
// touched by the lanes walking j's row, always the same lanes of the same
// wave; firstMessageDeliveries only by the lane owning receiver i.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "gsim_internal.h"
#include "philox.h"

namespace gsim {

// The member-major IHAVE walk reads a member's held / unseen window slots as two
// 128-bit masks (k_gossip_count_mm writes them) instead of one cell per slot, on
// sub-rings of at most kIhMaskSlots slots (0: the cells, for A/B builds)
#ifndef GSIM_IH_MASK
#define GSIM_IH_MASK 1
#endif
constexpr int kIhMaskSlots = 128;
__device__ __forceinline__ bool bit128(uint64_t w0, uint64_t w1, int k)
{
    return ((k < 64 ? w0 >> k : w1 >> (k - 64)) & 1ull) != 0;
}

// seen-set cell encoding: kUnseen64, kClaim, ... (gsim_internal.h)
constexpr int kMaxRing = 8192;     // active-slot list lives in LDS (u16, sized by the ring)

// The verdict of a message (gsim.h GSIM_VERDICT_*, stored in minv[slot]):
// any verdict but ACCEPT stops receivers from forwarding and putting it in
// their mcache; REJECT and SIGNATURE penalise every copy's sender (P4);
// SIGNATURE is rejected before markSeen, so its copies never claim a cell.
__device__ __forceinline__ bool verdict_penalises(uint8_t v)
{
    return v == GSIM_VERDICT_REJECT || v == GSIM_VERDICT_SIGNATURE;
}
#ifndef GSIM_SLOT_BATCH
#define GSIM_SLOT_BATCH 8
#endif
constexpr int kSlotBatch = GSIM_SLOT_BATCH;      // active slots whose cells are loaded together
// a shard's split commit: 4 topic groups, 4-slot batches per wave (serial K = 8
// C3 mean shard 11.80 / 11.78 ms against 11.91 / 11.87 with 8-slot batches; 8
// groups 12.12 / 12.16, 2 groups 11.80 / 11.77; 2-slot batches 11.91 / 11.89, 1-slot
// 12.08 / 12.02 against 11.83 / 11.84; profiles/r05_ab_summary.txt)
#ifndef GSIM_SPLIT_BATCH
#define GSIM_SPLIT_BATCH 4
#endif
#ifndef GSIM_SPLIT_GROUPS
#define GSIM_SPLIT_GROUPS 4
#endif
constexpr int kSplitBatch = GSIM_SPLIT_BATCH;    // ... per wave of a shard's split commit (k_commit<SPLIT>)
constexpr int kClSub = 64;
constexpr int kClStride = 32;       // u32s between two claim sub-list counters (own cache lines)
constexpr int kHubMesh = 16;       // mesh | direct edges listed per (hub, topic); more: the whole row is walked
constexpr uint32_t kHubList = 0x80000000u;   // k_send_tm s_beg flag: an offset into the hub lists         // claim sub-lists (block % kClSub): spreads the append atomics

// Validation latency (gsim_msg.vdelay).  A cell first
// claimed in round g of a slot with latency L > 0 is committed with
// hi = g + L, the round its validation completes; a copy arriving before
// that is a pending duplicate (deliveryUnknown, score.go:806-809), queued by
// its completion round and credited or penalised at the start of that round
// (k_vq_apply: score.go:719-725, 784-789), when the winner's
// markFirstMessageDelivery lands too; k_vcomplete at the end of round g + L
// sets the fresh bits (forwarding in round g + L + 1) and the mcache puts.
constexpr int kVqPlanes = GSIM_MAX_VDELAY + 1;   // queues by completion round mod kVqPlanes
constexpr uint32_t kVqFirst = 1, kVqDup = 2, kVqInv = 3;
// each plane's queue is kVqSub sub-lists (vq_cap / kVqSub entries) whose
// counters sit kVqStride u32s apart (own cache lines: append contention)
constexpr int kVqSub = 16, kVqStride = 32;
__host__ __device__ constexpr int64_t vq_ctr(int pl, int sub) { return ((int64_t)pl * kVqSub + sub) * kVqStride; }
constexpr int64_t kVqOver = (int64_t)kVqPlanes * kVqSub * kVqStride;   // overflow flag
constexpr int64_t kVqnWords = kVqOver + kVqStride;
static_assert((kVqPlanes & (kVqPlanes - 1)) == 0, "power-of-two planes");

struct Deliver {
    gsim_msg_config cfg{};
    uint32_t *d_mtopic = nullptr, *d_morigin = nullptr;
    uint8_t* d_minv = nullptr;
    uint8_t* d_mlat = nullptr;         // [ring] validation latency of the slot's message (gsim_msg.vdelay)
    uint64_t* d_vq = nullptr;          // [kVqPlanes][vq_cap] copies pending validation, by completion round
    uint8_t* d_vpc = nullptr;          // dense layout: [2][kVqPlanes][T * E] pending duplicate / invalid counts per record
    uint32_t* d_vqn = nullptr;         // sub-list counters (vq_ctr), then the overflow flag (kVqOver)
    uint32_t* d_hist = nullptr;        // [kVqPlanes][ring/32] slots with new claims, by round
    int64_t vq_cap = 0;
    bool lat_on = false;               // a message with vdelay > 0 was published
    uint64_t* d_mid = nullptr;         // [ring] gsim_msg.id of the slot's message (wire ids)
    uint64_t* d_cell = nullptr;        // seen-set cells (layout above; gsim_internal.h Cells)
    size_t n_cells = 0;
    uint64_t* d_cbase = nullptr;       // [ring] first cell of each slot
    std::vector<uint64_t> cbase;       // host copy
    uint64_t* d_mbits = nullptr;       // [T][nw] members of each topic (peers with its slot, §2)
    uint32_t* d_mpre = nullptr;        // [T][nw] members before each word
    uint64_t sparse = 0;               // topics with member-compacted cells (Cells::sparse)
    // member-major gossip (sub-rings with member-compacted cells): each topic's
    // members in peer order, so the IHAVE passes walk a topic's members, not N
    uint32_t* d_mlist = nullptr;       // members of the sparse topics, concatenated
    int64_t* d_mloff = nullptr;        // [T] first entry of each topic (-1: every peer, member j = peer j)
    int64_t* d_mcount = nullptr;       // [T] members of each topic
    uint32_t* d_mmtab = nullptr;       // [T+1] first 256-member block of each topic (k_ihave<MM>)
    uint32_t* d_hubw = nullptr;        // [hubw_cap] k_ihave<MM>'s waves with hub rows, then [1] their count
    int64_t hubw_cap = 0;
    uint32_t* d_mctab = nullptr;       // [T+1] first 1024-member block of each topic (k_gossip_count_mm)
    std::vector<uint32_t> mmtab, mctab;
    // member-major gossip on sub-rings of at most 128 slots: per member of each topic, the
    // window slots it holds and the ones it has not seen, by sub-ring index (k_gossip_count_mm)
    uint64_t* d_ihm = nullptr;         // [members][4]: held words 0-1, unseen words 2-3
    int64_t* d_mmb = nullptr;          // [T] first member of each topic in d_ihm
    int64_t cell_nw = 0;               // words per topic of the member bitmaps
    int64_t n_peers = 0;               // peers the cells were laid out for
    std::vector<int64_t> tcount;       // [T] messages published per topic (sub-ring slot choice)
    // publications per topic of the last kPubTicks ticks (ring by tick), for the
    // bound on a record's pending meshd increments (RoundArgs::mcnt_fast)
    std::vector<int32_t> pubw;         // [kPubTicks][T]
    std::vector<int64_t> pubw_tick;    // [kPubTicks] the tick each row counts
    int32_t pub_bound = 0;             // max over topics of the window's publications
    int64_t applied_tick = 0;          // tick of the last application of the pending increments
    uint32_t* d_pslot = nullptr;       // [pub_cap] ring slots of a publish batch
    gsim_msg* d_sched = nullptr;       // [sched_cap] gsim_step's publications, uploaded once per call
    uint32_t* d_sslot = nullptr;       // [sched_cap] ... and their ring slots
    int64_t sched_cap = 0;
    // claim list (member-compacted cells): the cells a round claimed, so the
    // commit touches those alone instead of every (active slot, peer word)
    uint64_t* d_clist = nullptr;       // [kClSub][clist_cap] receiver | slot << 32, in sub-lists
    uint32_t* d_clist_n = nullptr;     // [kClSub] entries, [kClSub] overflow (the commit then scans every word);
                                       // counter q at q * kClStride (one cache line each)
    int64_t clist_cap = 0;             // per sub-list
    // forwarder lists (list-driven send, k_send_list): the commit of round g-1
    // and the publications of round g-1 list round g's forwarders, so a sparse
    // round walks them instead of scanning every slot's fresh bits
    uint64_t* d_flist = nullptr;       // [2][flist_cap] by the send round's parity: peer | slot << 32 | origin << 63
    uint32_t* d_fst = nullptr;         // [kFstBad + p]: the list of parity p is incomplete; [p * kFstStride]: entries
    int64_t flist_cap = 0;
    int64_t flist_round = -1;          // the send round whose forwarders only the list holds (no fresh bits)
    uint64_t* d_seenbm = nullptr;      // [ring][ceil(N/64)] bit: the cell is committed (a cache of the cells)
    uint64_t* d_fresh = nullptr;       // [ring][ceil(N/64)] bit: the peer forwards the slot's message next round
    uint64_t* d_fsum = nullptr;        // [ring][ceil(N/4096)] bit: that fresh word may be non-zero
    uint64_t* d_mmask = nullptr;       // [T][N] mesh | direct positions of rows <= 64 (RoundArgs::mmask)
    // hub rows (> 64 connections): per (hub, topic) the row edges that are mesh
    // or direct, so a forwarding hub walks those few edges, not its whole row
    uint32_t* d_hidx = nullptr;        // [N] hub index of each row (~0: a row of at most 64)
    uint32_t* d_hrow = nullptr;        // [nhub] the hubs' rows
    uint32_t* d_hlist = nullptr;       // [nhub][T][1 + kHubMesh] count (~0: more) then the edges
    int64_t nhub = 0;
    int64_t hub_round = -1;            // round the lists were last built for (-1: stale)
    uint64_t mask_version = 0;         // h->mesh_version the masks were built for
    uint32_t* d_tmtab = nullptr;       // k_send_tm blocks: [T+1] first block of each topic, [T] its range
    std::vector<uint32_t> tmtab;       // host copy (the upload's source)
    int64_t tm_cn = -1;                // peers the table was built for
    int32_t tm_tb = 0;                 // k_send_tm block size d_tmtab was laid out for
    int32_t* d_mpub = nullptr;         // [ring] round the slot's message was published in
    int64_t* d_roff = nullptr;         // [rounds] offset of each round in its heartbeat
    int32_t* d_lastput = nullptr;      // [T][N]
    uint32_t* d_nnew = nullptr;        // [2][ring/32] bitmask: slots with new claims (or a publication), by round parity
    unsigned long long* d_stats = nullptr;   // [kStatLanes][kStatStride]: 4 totals per lane (stats_add)
    uint32_t* d_seen32 = nullptr;      // scratch for the F_SEEN view
    gsim_msg* d_pub = nullptr;
    int32_t pub_cap = 0;
    int64_t next_round = -1;           // -1: any
    int64_t pending = -1;              // round whose claims are not committed yet
    bool lazy = true;                  // every window >= 0: commits may trail a round
    // gossip
    int32_t* d_slot_last = nullptr;    // [ring] last round with a new claim or the publication
    uint8_t* d_gsel = nullptr;         // [T][E] sender edge order: emitGossip chose col[e] this heartbeat
    uint32_t* d_gcount = nullptr;      // [2][ring] holders / wanting receivers per slot (direction choice)
    uint8_t* d_gstate = nullptr;       // [E] edge order: owner's snapshot score of col >= gossipThreshold
    uint64_t* d_resp = nullptr;        // IWANT responses (record edge | slot << 32), delivered in round 2
    uint32_t* d_nresp = nullptr;       // [0] responses queued; [1] overflow; [2] ring-reuse error;
                                       // [3] bit 2: the gossip window exceeds MaxIHaveLength (k_ihave_pairs)
    uint8_t* d_peertx = nullptr;       // [ring][ptx_w] GetForPeer counts of bad-signature slots (IhArgs::peertx)
    int32_t ptx_w = 0;                 // longest local row
    int64_t resp_cap = 0;
    uint32_t* d_prom = nullptr;        // [P][E] promise ring, edge order of the promiser: slot or none
    uint64_t* d_pcand = nullptr;       // [E] per-IWANT promise candidate (min Philox key | slot)
    uint8_t* d_behaviour = nullptr;    // [N] GSIM_BEHAVE_*
    unsigned long long* d_gstats = nullptr;   // [4] gossip totals (gsim_gossip_stats)
    int32_t prom_ticks = 1;            // P
    std::vector<int64_t> prom_made;    // [P] tick that filled each ring index, -1 = empty
    int64_t ihave_tick = -1;           // heartbeat whose IHAVE marks are pending
    int64_t resp_round = -1;           // round in which the queued responses arrive
};

struct RoundArgs {
    int64_t N, E;
    int32_t T, ring, R;
    int64_t t0, hb, g, now;
    const uint32_t *row_ptr, *col;
    const uint8_t* dstate;     // GSIM_DS_* per edge index (router connected; record accept/tracked)
    const uint64_t* smask;     // topic slots of each row owner (nullptr: dense; gsim_internal.h)
    const uint32_t* owner;     // row owner of each edge index
    const uint8_t* mflags;     // router mesh bits, edge order
    const uint8_t* tflags;     // score bits, record order
    const gsim_topic_score_params* tp;
    double *first, *meshd, *invalid;
    uint8_t* mcnt;             // pending meshd increments, record order
    uint32_t *mtopic, *morigin;
    uint8_t* minv;
    uint64_t* mid;             // [ring] gsim_msg ids (wire ids)
    const uint8_t* mlat;       // [ring] validation latency (nullptr: none published, every latency 0)
    uint8_t* mlat_w;           // the same array, written by k_publish
    uint64_t* vq;              // [kVqPlanes][vq_cap] pending copies (Deliver::d_vq)
    uint8_t* vpc;              // Deliver::d_vpc (nullptr: every pending copy is a queue entry)
    int64_t vpe;               // records per plane of vpc (T * E)
    uint32_t* vqn;
    int64_t vq_cap;
    Cells cs;                  // the seen-set cells (gsim_internal.h)
    uint64_t* seenbm;          // [ring][nw] committed bits of the cells (read before a cell)
    uint64_t* fresh;           // [ring][nw] forwarders of the next round (topic-major delivery; nullptr otherwise)
    uint64_t* fsum;            // [ring][nsw] summary: bit j of word s = fresh word 64 s + j may be non-zero
    int64_t nw;                // words per slot
    int64_t nsw;               // summary words per slot
    int32_t* mpub;             // [ring] publication round
    const int64_t* roff;       // [R] (r + 1) * hb / (R + 1): offset of round r in its heartbeat
    int32_t* lastput;
    const uint32_t* nnew_prev;     // bitmask: slots with new claims (or a publication) in round g-1
    uint32_t* nnew_cur;            // bitmask: slots with new claims in round g
    unsigned long long* stats;
    int32_t* slot_last;
    uint32_t* err;                 // [0] responses queued, [1] overflow, [2] ring slot reused too early
    int32_t reuse_guard;           // rounds a slot must stay unpublished after its last activity
    // the origin's own Publish (gossipsub.go:989-1028): flood, mesh or fanout
    const uint64_t* sub;
    const double* score;           // snapshot, record order (flood publish filter)
    const uint32_t* rev;
    int32_t flood;
    double pub_thr;
    // every local peer may hold cells (a shard's ghost cells hold the
    // first-seen rounds their owners exported)
    int64_t CN;
    // receivers: the owned peers [rlo, rhi) (every peer unless sharded); a
    // shard pulls the copies its ghost senders forward to them, and leaves
    // the copies its own senders forward to ghosts to the ghosts' shards
    uint32_t rlo, rhi;
    int32_t sharded;
    const uint8_t* pgate;          // sharded flood publish: a ghost origin's score of the receiver >= publishThreshold
    // sharded: the edges of each row into owned peers (the copies this shard
    // delivers), a CSR of edge indices: row x's are sedge[sptr[x] .. sptr[x+1])
    const uint32_t *sptr, *sedge;
    // sharded, copy push: a copy of slot m on cross edge e sets
    // bit xwq[e] of row m of xbits ([ring][xbw] words: per destination shard a
    // word-aligned segment, bit = the edge's position in the cross-out list)
    int32_t push;
    int64_t slo, shi;              // k_send_tm's senders: [slo, shi) (slo a multiple of its chunk)
    const uint32_t* xwq;
    uint64_t* xbits;
    int64_t xbw;
    // [T][n] rows of at most 64 connections: bit q = row position q is a mesh or
    // direct edge (to an owned peer); a forwarder other than the origin sends
    // on no other edge, so only these are walked
    const uint64_t* mmask;
    const uint32_t *hidx, *hlist;  // hub rows' mesh edge lists (Deliver::d_hlist; nullptr: none)
    const uint32_t* tmtab;         // k_send_tm blocks per topic (Deliver::d_tmtab)
    uint8_t* peertx;               // [ring][ptx_w] GetForPeer counts (Deliver::d_peertx), zeroed on reuse
    int32_t ptx_w;
    TraceRef tr;                   // gsim_trace_config
    uint64_t* clist;               // claim list (Deliver::d_clist; nullptr: commits scan the words)
    int32_t cl_j;                  // entries carry the cell's member offset (cl_pack), else peer | slot << 32
    int32_t fl_from;               // forwarder entries carry the first sender (fl_entry), else peer | slot << 32
    uint32_t* clist_n;
    int64_t clist_cap;
    int64_t ncells;                // cells of the seen-set (the last slot's end)
    int32_t topic_slots;           // sub-rings: slots [t R, t R + R) carry topic t (0: one shared ring)
    // no record can collect 256 - 56 pending increments before the next refresh
    // (a record gets at most 1 + GossipRetransmission copies of a message, and
    // only of a message published in the last kPubTicks ticks): listed copies
    // add theirs without a returned value, no spill (atomic_mcnt_inc)
    int32_t mcnt_fast;
    // forwarder lists (Deliver::d_flist; nullptr: the fresh bits alone); flist_commit:
    // the commit lists its forwarders instead of setting fresh bits
    uint64_t* flist;
    uint32_t* fst;
    int64_t flist_cap;
    int32_t flist_commit;
    int32_t flist_send;            // k_send_tm: the list drives this round unless incomplete
    GaterRef gt;                   // peer gater (gater.hip; gt.act == nullptr: off)
    int32_t subdyn;                // a Leave happened: a receiver drops copies of topics it left
    uint32_t* inv_live;            // the invalid-plane flag the next refresh reads (inv_mark)
};

// The delivery totals: a block adds its 4 counts to one of kStatLanes
// cache-line-padded copies (by block index), so the thousands of blocks of a
// launch do not queue on 4 addresses; gsim_msg_stats sums the lanes.
constexpr int kStatLanes = 64, kStatStride = 16;
__device__ __forceinline__ void stats_add(const RoundArgs& a, unsigned long long acc, unsigned long long first,
                                          unsigned long long gray)
{
    unsigned long long* s = a.stats + (size_t)(blockIdx.x & (kStatLanes - 1)) * kStatStride;
    atomicAdd(&s[0], acc);
    atomicAdd(&s[1], first);
    atomicAdd(&s[2], acc - first);
    atomicAdd(&s[3], gray);
}

// A copy raised an invalidMessageDeliveries counter: the next refresh must
// read that plane (engine.hip k_refresh_score skips it while the flag is 0)
__device__ __forceinline__ void inv_mark(const RoundArgs& a)
{
    if (a.inv_live && !__hip_atomic_load(a.inv_live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        __hip_atomic_store(a.inv_live, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The peer gater's AcceptFrom (peer_gater.go:320-363) at receiver i for a
// copy from sender j, record r (i's record of j: its stats group gq[r]),
// slot m: true = AcceptAll.  rand.Float64() is a Philox uniform keyed by
// (round, receiver, slot | P_GATER, sender) (oracle_gater.c).  AcceptControl
// drops the message and runs ThrottlePeer (gossip_tracer.go:182-200): i's
// promises from j are forgotten.  Direct peers are accepted
// (gossipsub.go:599-602).
constexpr uint32_t kGaterRpcSlot = 0xFFFFFFu;   // the draw key of an IWANT answer (oracle ORC_GATER_RPC_SLOT)

__device__ __forceinline__ bool gater_accept(const RoundArgs& a, uint32_t i, uint32_t r, uint32_t m, uint32_t j)
{
    const GaterRef& g = a.gt;
    if (!g.act[i]) return true;
    const uint32_t ei = a.rev[r];                          // i's edge to j
    if (g.direct && g.direct[ei]) return true;
    const uint32_t q = g.gq[r];
    const double del = g.del[q];
    const double total = del + g.dw * g.dup[q] + g.iw * g.ign[q] + g.rw * g.rej[q];
    if (total == 0) return true;
    const double thr = (1 + del) / (1 + total);
    // (a shard: the draw keys on global ids, as the single engine's)
    const uint32_t ig = g.gid ? g.gid[i] : i, jg = g.gid ? g.gid[j] : j;
    const u32x4 x = philox4x32_10((uint32_t)a.g, ig, (m << 8) | P_GATER, jg, (uint32_t)g.seed, (uint32_t)(g.seed >> 32));
    const uint64_t r53 = ((uint64_t)x.x << 21) | (x.y >> 11);
    if ((double)r53 * (1.0 / 9007199254740992.0) < thr) return true;
    for (int32_t q2 = 0; q2 < g.P; ++q2) g.prom[(int64_t)q2 * a.E + ei] = 0xFFFFFFFFu;
    atomicAdd(g.n_thr, 1ull);
    return false;
}

// a copy the receiver handled: DuplicateMessage, or the bad signature's
// RejectMessage (peer_gater.go:393-432); the claim winner is converted at commit
__device__ __forceinline__ void gater_copy(const RoundArgs& a, uint32_t r, bool sig)
{
    const uint32_t q = a.gt.gq[r];
    atomicAdd(sig ? &a.gt.a_rej[q] : &a.gt.a_dup[q], 1u);
}

// the first delivery of record r at receiver i: ValidateMessage and the
// verdict's Deliver/RejectMessage instead of a duplicate
__device__ __forceinline__ void gater_first(const RoundArgs& a, uint32_t r, uint32_t i, int32_t t, uint8_t verdict)
{
    const GaterRef& g = a.gt;
    const uint32_t q = g.gq[r];
    atomicSub(&g.a_dup[q], 1u);
    atomicAdd(&g.a_val[i], 1u);
    if (verdict == GSIM_VERDICT_ACCEPT) {
        atomicAdd(&g.a_del[q], g.tw[t]);
    } else if (verdict == GSIM_VERDICT_REJECT) {
        atomicAdd(&g.a_rej[q], 1u);
    } else if (verdict == GSIM_VERDICT_IGNORE) {
        atomicAdd(&g.a_ign[q], 1u);
    } else if (verdict == GSIM_VERDICT_THROTTLE) {
        atomicAdd(&g.a_thr[i], 1u);
        g.a_last[i] = 1;
    }
}

__device__ __forceinline__ int64_t round_time(const RoundArgs& a, int64_t g)
{
    // T(g) = t0 + (g / R) * hb + (g % R + 1) * hb / (R + 1): rounds fit in 31
    // bits, and the last term is a table (32-bit division, no 64-bit one)
    const uint32_t q = (uint32_t)g / (uint32_t)a.R;
    const uint32_t r = (uint32_t)g - q * (uint32_t)a.R;
    return a.t0 + (int64_t)q * a.hb + a.roff[r];
}

// lanes of group `grp` when a wave is split into groups of W lanes
template <int W>
__device__ __forceinline__ uint64_t group_mask(int grp)
{
    if constexpr (W == 64) return ~0ull;
    else return ((1ull << W) - 1) << (grp * W);
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// x -> min(x + 1, cap) on a counter other lanes may update concurrently
// (only the negative-window P3 credit of a first delivery needs it).
__device__ __forceinline__ void atomic_inc_capped(double* p, double cap)
{
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    unsigned long long old = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        double x = __longlong_as_double((long long)old) + 1.0;
        if (x > cap) x = cap;
        const unsigned long long nw = (unsigned long long)__double_as_longlong(x);
        if (nw == old) return;
        const unsigned long long prev = atomicCAS(q, old, nw);
        if (prev == old) return;
        old = prev;
    }
}

// Queue a copy whose receiver completes validation in round c: record edge
// e of topic t (score records sit at the sender's edge index), and what the
// completion does with it (kVqFirst / kVqDup / kVqInv).
__device__ __forceinline__ void vq_push(const RoundArgs& a, int64_t c, uint32_t e, int32_t t, uint32_t kind)
{
    const int pl = (int)(c & (kVqPlanes - 1));
    const int sub = (int)((blockIdx.x + (threadIdx.x >> 6)) % kVqSub);
    const int64_t scap = a.vq_cap / kVqSub;
    const uint32_t k = atomicAdd(&a.vqn[vq_ctr(pl, sub)], 1u);
    if ((int64_t)k >= scap) { atomicOr(&a.vqn[kVqOver], 1u); return; }
    a.vq[(int64_t)pl * a.vq_cap + sub * scap + k] = (uint64_t)e | ((uint64_t)(uint32_t)t << 32) | ((uint64_t)kind << 40);
}

// vq_push for a whole wave from convergent code: lane entries with pl >= 0
// go to plane pl, one queue atomic per distinct plane in the wave.
__device__ __forceinline__ void vq_push_wave(const RoundArgs& a, int pl, uint64_t v)
{
    const int lane = threadIdx.x & 63;
    const int sub = (int)((blockIdx.x * 16u + (threadIdx.x >> 6)) % kVqSub);
    const int64_t scap = a.vq_cap / kVqSub;
    uint64_t pending = __ballot(pl >= 0);
    while (pending) {
        const int leader = __builtin_ctzll(pending);
        const int lpl = __shfl(pl, leader, 64);
        const uint64_t grp = __ballot(pl == lpl) & pending;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&a.vqn[vq_ctr(lpl, sub)], (uint32_t)__popcll(grp));
        base = (uint32_t)__shfl((int)base, leader, 64);
        if (pl == lpl) {
            const uint32_t k = base + (uint32_t)__popcll(grp & ((1ull << lane) - 1));
            if ((int64_t)k < scap) a.vq[(int64_t)lpl * a.vq_cap + sub * scap + k] = v;
            else atomicOr(&a.vqn[kVqOver], 1u);
        }
        pending &= ~grp;
    }
}

__device__ __forceinline__ uint64_t vq_entry(uint32_t e, int32_t t, uint32_t kind)
{
    return (uint64_t)e | ((uint64_t)(uint32_t)t << 32) | ((uint64_t)kind << 40);
}

// Append the lanes' new claims (receiver | slot << 32) to the block's claim
// sub-list, one atomic per wave; every lane of the wave calls it.
// A claim-list entry.  Packed (RoundArgs::cl_j, peers < 2^24): peer i (24 bits), slot m
// (13), the claimed cell's offset in the slot (27): the commit finds the cell from
// cbase[m] alone, not through the member tables (one random trip less per claim).
#ifndef GSIM_CL_PACK
#define GSIM_CL_PACK 1
#endif
constexpr uint32_t kClPeerMax = 1u << 24;
__device__ __forceinline__ uint64_t cl_entry(const RoundArgs& a, uint32_t i, uint32_t m, int64_t ci, int64_t cb)
{
    return a.cl_j ? (uint64_t)i | ((uint64_t)m << 24) | ((uint64_t)(ci - cb) << 37) : (uint64_t)i | ((uint64_t)m << 32);
}
__device__ __forceinline__ void clist_push_wave(const RoundArgs& a, bool on, uint64_t v)
{
    const uint64_t b = __ballot(on);
    if (!b) return;
    const int lane = threadIdx.x & 63, leader = __builtin_ctzll(b);
    const uint32_t q = blockIdx.x % kClSub;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&a.clist_n[q * kClStride], (uint32_t)__popcll(b));
    base = (uint32_t)__shfl((int)base, leader, 64);
    if (on) {
        const uint32_t k = base + (uint32_t)__popcll(b & ((1ull << lane) - 1));
        if ((int64_t)k < a.clist_cap) a.clist[(int64_t)q * a.clist_cap + k] = v;
        else atomicOr(&a.clist_n[kClSub * kClStride], 1u);
    }
}

// Slots of word w (bits) got a new claim in round g: their activity bit and
// last-active round.  Every block of a launch reports the slots it touched,
// and same-address atomics serialise (thousands of blocks on ~40 slots), so a
// value already there -- a load returns it or an older one, both only grow
// within the round -- is not written again.
__device__ __forceinline__ void slots_claimed(const RoundArgs& a, int w, uint32_t bits)
{
    const uint32_t have = __hip_atomic_load(&a.nnew_cur[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((have & bits) != bits) atomicOr(&a.nnew_cur[w], bits);
    while (bits) {
        const int q = __ffs(bits) - 1;
        bits &= bits - 1;
        int32_t* sl = &a.slot_last[w * 32 + q];
        if (__hip_atomic_load(sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (int32_t)a.g) atomicMax(sl, (int32_t)a.g);
    }
}

// Mark fresh bits of word w of slot m (and the word in the summary).
__device__ __forceinline__ void fresh_set(const RoundArgs& a, uint32_t m, int64_t w, uint64_t bits)
{
    atomicOr(reinterpret_cast<unsigned long long*>(a.fresh + (int64_t)m * a.nw + w), bits);
    uint64_t* sp = a.fsum + (int64_t)m * a.nsw + (w >> 6);
    const uint64_t sb = 1ull << (w & 63);
    if (!(__hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & sb))
        atomicOr(reinterpret_cast<unsigned long long*>(sp), sb);
}

// Forwarder list state (Deliver::d_fst): entries of parity p at p * kFstStride
// (own cache lines), the incomplete flag of parity p at kFstBad + p
constexpr int kFstStride = 32;
constexpr int kFstBad = 2 * kFstStride;
constexpr uint64_t kFlOrigin = 1ull << 63;
// A forwarder entry.  Packed (RoundArgs::fl_from, peers < 2^24 - 1): forwarder x (24
// bits), slot m (13), its first sender (24; kFlNone: none), origin flag (bit 63): the
// send reads the sender from the entry, not from the forwarder's committed cell
// (the member tables, then the cell: two random trips per forwarder).
#ifndef GSIM_FL_PACK
#define GSIM_FL_PACK 1
#endif
constexpr uint32_t kFlNone = (1u << 24) - 1u;
__device__ __forceinline__ uint64_t fl_entry(const RoundArgs& a, uint32_t x, uint32_t m, uint32_t from)
{
    if (!a.fl_from) return (uint64_t)x | ((uint64_t)m << 32);
    const uint32_t f = from < kFlNone ? from : kFlNone;
    return (uint64_t)x | ((uint64_t)m << 24) | ((uint64_t)f << 37);
}
__device__ __forceinline__ uint32_t fl_x(const RoundArgs& a, uint64_t v) { return a.fl_from ? (uint32_t)(v & kFlNone) : (uint32_t)v; }
__device__ __forceinline__ uint32_t fl_m(const RoundArgs& a, uint64_t v)
{
    return a.fl_from ? (uint32_t)((v >> 24) & 0x1FFFu) : (uint32_t)(v >> 32) & 0x7FFFFFFFu;
}
__device__ __forceinline__ uint32_t fl_from_of(uint64_t v)
{
    const uint32_t f = (uint32_t)((v >> 37) & kFlNone);
    return f == kFlNone ? kPeerMask : f;
}

// Append the lanes' forwarders (on, peer | slot << 32) of send round g to its
// list; every lane of the wave calls it.  An entry that does not fit marks
// the list incomplete and becomes a fresh bit; the send then converts the
// entries that fit (k_flist_fresh) and scans the bits (k_send_tm), so no
// forwarder is lost however the lists are sized (gsim_msg_config.max_frontier).
__device__ __forceinline__ void flist_push_wave(const RoundArgs& a, int64_t g, bool on, uint64_t v)
{
    const uint64_t b = __ballot(on);
    if (!b) return;
    const int lane = threadIdx.x & 63, leader = __builtin_ctzll(b), p = (int)(g & 1);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&a.fst[p * kFstStride], (uint32_t)__popcll(b));
    base = (uint32_t)__shfl((int)base, leader, 64);
    if (on) {
        const uint32_t k = base + (uint32_t)__popcll(b & ((1ull << lane) - 1));
        if ((int64_t)k < a.flist_cap) {
            a.flist[(int64_t)p * a.flist_cap + k] = v;
        } else {
            a.fst[kFstBad + p] = 1;
            const uint32_t x = fl_x(a, v), m = fl_m(a, v);
            fresh_set(a, m, (int64_t)(x >> 6), 1ull << (x & 63));
        }
    }
}

// Ordered list of the active slots (bit set in nnew), built by wave 0 into
// LDS; every thread of the block must call it.
__device__ __forceinline__ int active_slots(const uint32_t* nnew, int ring, uint16_t* s_act, int* s_n)
{
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        int n = 0;
        for (int m0 = 0; m0 < ring; m0 += 64) {
            const int m = m0 + lane;
            const bool act = m < ring && ((nnew[m >> 5] >> (m & 31)) & 1u);
            const uint64_t b = __ballot(act);
            if (act) s_act[n + __popcll(b & ((1ull << lane) - 1))] = (uint16_t)m;
            n += __popcll(b);
        }
        if (lane == 0) *s_n = n;
    }
    __syncthreads();
    return *s_n;
}

// The active slots of topics t with t % ngrp == grp (the split commit's share:
// slots of different topics never credit the same record or lastput word).
__device__ __forceinline__ int active_slots_topics(const uint32_t* nnew, int ring, const uint32_t* mtopic, int grp,
                                                   int ngrp, uint16_t* s_act, int* s_n)
{
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        int n = 0;
        for (int m0 = 0; m0 < ring; m0 += 64) {
            const int m = m0 + lane;
            const bool act = m < ring && ((nnew[m >> 5] >> (m & 31)) & 1u) && (int)(mtopic[m] % (uint32_t)ngrp) == grp;
            const uint64_t b = __ballot(act);
            if (act) s_act[n + __popcll(b & ((1ull << lane) - 1))] = (uint16_t)m;
            n += __popcll(b);
        }
        if (lane == 0) *s_n = n;
    }
    __syncthreads();
    return *s_n;
}

// Commit one claimed cell of round gc (markSeen + the winner's P2/P3 credit,
// markFirstMessageDelivery score.go:919-946; mcache.Put for lastput).
template <bool ATOMIC = false, bool LAT = false, bool SP = true, bool GT = false>
__device__ __forceinline__ void commit_claim(const RoundArgs& a, uint64_t* cellp, uint64_t c, int64_t gc,
                                             uint32_t m, int64_t peer, int* qpl = nullptr, uint64_t* qv = nullptr)
{
    const uint32_t hi = (uint32_t)(c >> 32), lo = (uint32_t)c;
    if constexpr (LAT) {
        const uint32_t L = a.mlat[m];
        *cellp = ((uint64_t)(uint32_t)(gc + L) << 32) | (lo & kPeerMask);
        if (L) {
            // validation completes in round gc + L: the winner's DeliverMessage
            // credit lands there (k_vq_apply), the put and forwarding after it
            const int32_t t = (int32_t)a.mtopic[m];
            if (a.minv[m] == GSIM_VERDICT_ACCEPT && const_tp(a.tp)[t].scored) {
                if (qpl) {                                  // k_commit pushes per wave
                    *qpl = (int)((gc + L) & (kVqPlanes - 1));
                    *qv = vq_entry(hi & kEdgeMask, t, kVqFirst);
                } else {
                    vq_push(a, gc + L, hi & kEdgeMask, t, kVqFirst);
                }
            }
            return;
        }
    } else {
        *cellp = ((uint64_t)(uint32_t)gc << 32) | (lo & kPeerMask);
    }
    if constexpr (GT) gater_first(a, hi & kEdgeMask, (uint32_t)peer, (int32_t)a.mtopic[m], a.minv[m]);
    if (a.minv[m]) return;                                // RejectMessage: counted when sent
    const int32_t t = (int32_t)a.mtopic[m];
    int32_t* lp = a.lastput + (int64_t)t * a.N + peer;
    const int32_t tick = (int32_t)(gc / a.R);
    if (ATOMIC) atomicMax(lp, tick); else if (*lp < tick) *lp = tick;
    if (!(lo & kCreditFirst)) return;
    const ctp_t tp = const_tp(a.tp) + t;
    // the winner's record sits at its edge, in the sender's row (its topic slot)
    const int64_t ir = SP ? slot_idx(smask_of(a.smask, lo & kPeerMask), t, a.E, hi & kEdgeMask)
                          : (int64_t)t * a.E + (hi & kEdgeMask);
    const double cap = tp->first_message_deliveries_cap;
    if (ATOMIC) {
        atomic_inc_capped(&a.first[ir], cap);
    } else {
        const double x = a.first[ir] + 1.0;
        a.first[ir] = x > cap ? cap : x;
    }
    // with a negative window no same-round copy was credited; the first
    // delivery is credited regardless of the window
    if (lo & kCreditMesh) atomic_inc_capped(&a.meshd[ir], tp->mesh_message_deliveries_cap);
}

// Cell index of lane `lane` of the 64-peer word w in slot m (gsim_internal.h
// Cells): every lane of a wave asks for the same (m, w), so the slot's base
// and the topic's member word are wave-uniform loads; -1: no cell.
// SP = false: the dense layout (no sparse topic), m * n + p without a read.
template <bool SP>
__device__ __forceinline__ int64_t word_cell(const Cells& c, const uint32_t* mtopic, uint32_t m, int64_t w, int lane)
{
    if (!SP || !c.sparse) return (int64_t)m * c.n + w * 64 + lane;
    uint64_t bits;
    int64_t pre;
    c.word((int32_t)mtopic[m], w, bits, pre);
    const uint64_t bit = 1ull << lane;
    if (!(bits & bit)) return -1;
    return (int64_t)c.cbase[m] + pre + __popcll(bits & (bit - 1));
}

__device__ __forceinline__ bool is_claim_of(uint64_t c, uint32_t parity)
{
    const uint32_t hi = (uint32_t)(c >> 32);
    return c != kUnseen64 && (hi & kClaim) && ((hi >> 30) & 1u) == parity;
}


// Reset the cells and bitmaps of the slots being published into.  Every
// claim is committed before (gsim_publish flushes the last round), so the
// slot's cells — one contiguous range per slot — are simply made unseen.
__global__ void k_reset_slots(RoundArgs a, const uint32_t* pslot, int32_t count)
{
    const int k = blockIdx.y;
    if (k >= count) return;
    const uint32_t m = pslot[k];
    // the previous message may still sit in a gossip window or a promise
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.slot_last[m] >= 0 && a.g - a.slot_last[m] < a.reuse_guard)
        atomicOr(&a.err[2], 1u);
    if (blockIdx.x == 0 && a.peertx)
        for (int j = threadIdx.x; j < a.ptx_w; j += blockDim.x) a.peertx[(int64_t)m * a.ptx_w + j] = 0;
    const int64_t base = (int64_t)a.cs.cbase[m];
    const int64_t end = (int64_t)m + 1 < a.ring ? (int64_t)a.cs.cbase[m + 1] : a.ncells;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = base + tid; j < end; j += stride) a.cs.cell[j] = kUnseen64;
    for (int64_t w = tid; w < a.nw; w += stride) {
        a.seenbm[(int64_t)m * a.nw + w] = 0;
        if (a.fresh) a.fresh[(int64_t)m * a.nw + w] = 0;
    }
    if (a.fresh)
        for (int64_t w = tid; w < a.nsw; w += stride) a.fsum[(int64_t)m * a.nsw + w] = 0;
}

__global__ void k_publish(RoundArgs a, const gsim_msg* pub, const uint32_t* pslot, int32_t count)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    const gsim_msg p = pub[k];
    const uint32_t slot = pslot[k];
    a.mtopic[slot] = p.topic;
    a.morigin[slot] = p.origin;          // local id (a shard: 0xFFFFFFFF when not a local peer)
    a.minv[slot] = p.verdict;
    a.mlat_w[slot] = p.vdelay;
    a.mpub[slot] = (int32_t)a.g;
    if (a.mid) a.mid[slot] = p.id;
    const int64_t oci = (int64_t)p.origin < a.CN ? a.cs.idx(slot, (int32_t)p.topic, p.origin) : -1;
    if (oci >= 0) {                                        // the origin's own cell (it holds the topic, §2)
        const uint32_t oc = p.origin;
        a.cs.cell[oci] = ((uint64_t)(uint32_t)a.g << 32) | p.origin;
        atomicOr(reinterpret_cast<unsigned long long*>(a.seenbm + (int64_t)slot * a.nw + (oc >> 6)), 1ull << (oc & 63));
        // the origin publishes whatever the verdict (push: a ghost origin's own shard sends)
        if (a.fresh && (!a.push || (oc >= a.rlo && oc < a.rhi))) {
            fresh_set(a, slot, oc >> 6, 1ull << (oc & 63));
            if (a.flist) {                                 // ... and in round g+1's forwarder list
                const int pp = (int)((a.g + 1) & 1);
                const uint32_t q = atomicAdd(&a.fst[pp * kFstStride], 1u);
                if ((int64_t)q < a.flist_cap) a.flist[(int64_t)pp * a.flist_cap + q] = fl_entry(a, oc, slot, oc) | kFlOrigin;
                else a.fst[kFstBad + pp] = 1;
            }
        }
        int32_t* lp = a.lastput + (int64_t)p.topic * a.N + p.origin;
        const int32_t tick = (int32_t)(a.g / a.R);
        if (*lp < tick) *lp = tick;
    }
    atomicOr(&a.nnew_cur[slot >> 5], 1u << (slot & 31));   // the origin forwards in round g+1
    a.slot_last[slot] = (int32_t)a.g;
    if (a.tr.on(p.origin))                                  // PublishMessage (trace.go:70-91)
        a.tr.push(round_time(a, a.g), p.id, p.origin, p.origin, (int32_t)p.topic, GSIM_TRACE_PUBLISH_MESSAGE, 0);
}

// Position of the k-th set bit (k < popcount) of m.
__device__ __forceinline__ uint32_t kth_bit(uint64_t m, uint32_t k)
{
    uint32_t pos = 0;
#pragma unroll
    for (int w = 32; w; w >>= 1) {
        const uint64_t lo = m & ((1ull << w) - 1);
        const uint32_t c = (uint32_t)__popcll(lo);
        if (k >= c) { k -= c; m >>= w; pos += (uint32_t)w; } else { m = lo; }
    }
    return pos;
}

// The mesh masks of rows of at most 64 connections: bit q of mmask[t][x] =
// position q of row x carries the router's mesh bit for t, or is a direct
// peer; only edges to the receivers [rlo, rhi) (a shard's owned peers).
__global__ __launch_bounds__(256) void k_mesh_mask(const uint32_t* row_ptr, const uint32_t* col, const uint8_t* mflags,
                                                   const uint8_t* direct, const uint64_t* smask, int64_t n, int64_t E,
                                                   int32_t T, uint32_t rlo, uint32_t rhi, uint64_t* mmask,
                                                   int64_t row_lo, int64_t row_hi)
{
    // one wave per row of [row_lo, row_hi), lane = row position: coalesced flag planes, one ballot per topic
    const int lane = threadIdx.x & 63;
    for (int64_t r = row_lo + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < row_hi; r += (int64_t)gridDim.x * 4) {
        const uint32_t b = row_ptr[r], d = row_ptr[r + 1] - b;
        const bool v = d <= 64 && (uint32_t)lane < d;
        const uint32_t e = b + (uint32_t)lane;
        const uint32_t i = v ? col[e] : 0u;
        const bool own = v && i >= rlo && i < rhi;
        const bool dir = own && direct && direct[e];
        const uint64_t m = smask_of(smask, (uint32_t)r);
        for (int32_t t = 0; t < T; ++t) {
            const bool me = own && (dir || (slot_has(m, t) && (mflags[slot_idx(m, t, E, e)] & GSIM_TF_MESH)));
            const uint64_t m = __ballot(me);
            if (lane == 0) mmask[(int64_t)t * n + r] = m;
        }
    }
}

// The mesh lists of hub rows: per (hub, topic) the row edges to the receivers
// [rlo, rhi) that carry the router's mesh bit or are direct peers, in row
// order, one wave per hub (ballots over 64-position chunks).  More than
// kHubMesh such edges: count ~0, the hub walks its whole row for t.
constexpr int kHubBatch = 4;     // k_hub_mesh: topics whose flags a lane loads at once
__global__ __launch_bounds__(256) void k_hub_mesh(const uint32_t* row_ptr, const uint32_t* col, const uint8_t* mflags,
                                                  const uint8_t* direct, const uint64_t* smask, const uint32_t* hrow,
                                                  int64_t nhub, int64_t E, int32_t T, uint32_t rlo, uint32_t rhi,
                                                  uint32_t* hlist)
{
    const int lane = threadIdx.x & 63;
    for (int64_t hx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); hx < nhub; hx += (int64_t)gridDim.x * 4) {
        const uint32_t x = hrow[hx];
        const uint32_t b = row_ptr[x], d = row_ptr[x + 1] - b;
        const uint64_t m = smask_of(smask, x);
        uint32_t* const L0 = hlist + (int64_t)hx * T * (1 + kHubMesh);
        for (int32_t t = lane; t < T; t += 64)
            if (!slot_has(m, t)) L0[(int64_t)t * (1 + kHubMesh)] = 0;
        // the row is walked once for every topic the hub holds: a chunk's ends
        // and direct flags are loaded once, its topics' flags kHubBatch at a time;
        // lane t keeps topic t's count
        uint32_t cnt = 0;
        for (uint32_t off = 0; off < d; off += 64) {
            const uint32_t e = b + off + (uint32_t)lane;
            const bool v = off + (uint32_t)lane < d;
            const uint32_t i = v ? col[e] : 0u;
            const bool own = v && i >= rlo && i < rhi;
            const bool dr = own && direct && direct[e];
            for (uint64_t mm = m; mm;) {
                int tb[kHubBatch];
                uint8_t fb[kHubBatch];
#pragma unroll
                for (int q = 0; q < kHubBatch; ++q) {
                    tb[q] = mm ? __builtin_ctzll(mm) : -1;
                    if (mm) mm &= mm - 1;
                    fb[q] = (tb[q] >= 0 && own && !dr) ? mflags[slot_idx(m, tb[q], E, e)] : (uint8_t)0;
                }
#pragma unroll
                for (int q = 0; q < kHubBatch; ++q) {
                    const int t = tb[q];
                    if (t < 0) break;                                    // wave-uniform
                    const bool me = dr || (fb[q] & GSIM_TF_MESH);
                    const uint64_t bal = __ballot(me);
                    const uint32_t base = (uint32_t)__shfl((int)cnt, t, 64);
                    if (me) {
                        const uint32_t pos = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
                        if (pos < (uint32_t)kHubMesh) L0[(int64_t)t * (1 + kHubMesh) + 1 + pos] = e;
                    }
                    if (lane == t) cnt += (uint32_t)__popcll(bal);
                }
            }
        }
        if (lane < T && slot_has(m, lane))
            L0[(int64_t)lane * (1 + kHubMesh)] = cnt <= (uint32_t)kHubMesh ? cnt : 0xFFFFFFFFu;
    }
}

__global__ __launch_bounds__(256) void k_hub_index(const uint32_t* row_ptr, int64_t n, uint32_t* hidx, uint32_t* hrow,
                                                   uint32_t* count)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += stride) {
        uint32_t k = 0xFFFFFFFFu;
        if (row_ptr[x + 1] - row_ptr[x] > 64u) {
            k = atomicAdd(count, 1u);
            if (hrow) hrow[k] = (uint32_t)x;
        }
        if (hidx) hidx[x] = k;
    }
}

// Delivery round g, topic-major.  Block (range, topic)
// walks the forwarders of its peer range for every active slot of topic t.
// It takes each chunk of the range once and gathers there the forwarders of
// all the topic's active slots (64 slots per pass), so a round with many
// sparse slots (c5: a few forwarders per slot and chunk) walks one frontier
// per chunk, not one per slot and chunk.  Requires every claim of round g-1
// committed (k_commit runs first): the committed bits then hold every
// receiver seen before round g.
//
// Records a block updates — meshMessageDeliveries / invalid of the receivers'
// records about its senders (record order: the senders' rows), per topic —
// belong to this block alone.  A sender fresh in several slots of the topic
// would update them from several lanes at once, so its slots are taken in
// layers (layer l: each peer's l-th slot of the pass), one after the other.
// Results are identical to k_send's.
//
// A chunk's frontier is flattened into its edges: a prefix sum of the
// senders' walk lengths in LDS, one thread per edge (binary search for the
// edge's sender), so rows of any length keep every lane busy — a shard's
// short rows (owned rows cut to their owned receivers, ghost rows) as much as
// power-law hubs.  Forwarders walk their mesh mask (rows <= 64), the origin
// and hubs their whole row.
constexpr int kTsSlots = 64;
#ifndef GSIM_TM_P
#define GSIM_TM_P 2          // flattened edges per thread per iteration (loads interleaved)
#endif
#ifndef GSIM_TM_MINB
#define GSIM_TM_MINB 1       // waves per SIMD the register budget is fitted to
#endif
// threads per dense k_send_tm block, and its waves per SIMD: 512 threads at 6
// waves (80 VGPRs, 11 spilled; 3 blocks per CU) against 1024 at 4 (1 block): C3
// send 15.25 -> 13.56 ms per tick, 256 at 6: 15.68 (gpurun_out/r04ab2, one box).
// The walk waits on its dependent trips; more resident waves hide more of them.
#ifndef GSIM_TM_TB
#define GSIM_TM_TB 512
#endif
#ifndef GSIM_TM_MINB_DENSE
#define GSIM_TM_MINB_DENSE 6
#endif
#ifndef GSIM_TM_MINB_SPARSE
#define GSIM_TM_MINB_SPARSE 1
#endif
// (non-temporal loads of the row fields and cells, to keep the committed
// bitmaps in L2, were measured slower in round 4 and removed)
// a shard's push walk: 512-thread blocks fitted to 4 waves per SIMD (two blocks
// per CU), serial K = 8 C3 mean shard 11.66 / 11.67 -> 11.49 / 11.52 ms against
// 1024 threads at 4 waves (512 at 6 waves: 11.73 / 11.75; round 3: 512 at one
// wave 21 against 18.5 ms), gpurun_out/r05h_ab
#ifndef GSIM_TM_PUSH_TB
#define GSIM_TM_PUSH_TB 512
#endif
#ifndef GSIM_TM_MINB_PUSH
#define GSIM_TM_MINB_PUSH 4
#endif
constexpr int kPushTB = GSIM_TM_PUSH_TB;
// ... with member-compacted cells (sparse frontiers: many topics, each block's
// chunks hold few forwarders): c5 send 184 / 151 / 158 ms per tick at 1024 / 512 /
// 256 threads (gpurun_out/r04n); dense C3: GSIM_TM_TB (§4.2)
constexpr int kSparseTB = 512;
constexpr uint32_t kTmWin = 8192;   // flattened edges whose senders are tabled in LDS at once
// forwarders in a chunk from which the sender table pays for its fill: every chunk
// since the 1024-peer chunks of round 4 (C3 holds ~165 forwarders a layer): send
// 14.27 / 14.28 against 14.39 / 14.40 ms per tick at 256 (profiles/r05_ab_summary.txt)
#ifndef GSIM_TM_TAB_MIN
#define GSIM_TM_TAB_MIN 0
#endif
constexpr int kTmTabMin = GSIM_TM_TAB_MIN;

// The wave's remote copies as bits (copy push): lane l sets
// bits v of xbits word k (~0: none).  Neighbouring lanes carry neighbouring
// senders' copies, whose bits share words: an OR-scan over runs of equal
// words, and the run's last lane issues one atomicOr for all of them (a lane
// may also take in bits of an earlier run of the same word: OR is idempotent).
// Every lane of the wave calls it.
__device__ __forceinline__ void xbits_or_wave(uint64_t* xbits, uint64_t k, uint64_t v)
{
    const int lane = threadIdx.x & 63;
    if (!__ballot(k != ~0ull)) return;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t ko = (uint64_t)__shfl_up((long long)k, o, 64);
        const uint64_t vo = (uint64_t)__shfl_up((long long)v, o, 64);
        if (lane >= o && ko == k) v |= vo;
    }
    const uint64_t kn = (uint64_t)__shfl_down((long long)k, 1, 64);
    if (k != ~0ull && (lane == 63 || kn != k))
        atomicOr(reinterpret_cast<unsigned long long*>(xbits + k), (unsigned long long)v);
}

// Diagnostic build (-DGSIM_DIAG_PHASE, timing only): shader clocks per wave in
// k_send_tm's phases -- [0] all, [1] chunk scans and layer layouts, [2] edge
// walks, [3] waves, [4] layout + walk clocks of the layers after a chunk's
// first, [5] chunk-layers, [6] chunks with a frontier, [7] forwarders of the
// later layers (per block, summed by wave 0) -- over a launch (gsim_diag_send_phases)
#ifdef GSIM_DIAG_PHASE
__device__ unsigned long long g_tm_diag[8];
#define TM_CLK(v) const unsigned long long v = (unsigned long long)clock64()
#define TM_ACC(d, a, b) d += (b) - (a)
#else
#define TM_CLK(v)
#define TM_ACC(d, a, b)
#endif

// SP: topic slots or member-compacted cells are in use (gsim_internal.h); the
// dense instance indexes plane t and cell m * N + p with no table reads.
template <int kTmThreads, bool LAT, bool SP, bool GT = false, bool PUSH = false>
__global__ __launch_bounds__(kTmThreads, PUSH ? GSIM_TM_MINB_PUSH
                                        : (!SP && kTmThreads == GSIM_TM_TB) ? GSIM_TM_MINB_DENSE
                                        : (SP && !LAT && kTmThreads == kSparseTB) ? GSIM_TM_MINB_SPARSE
                                                                                   : GSIM_TM_MINB)
void k_send_tm(RoundArgs a_)
{
    const RoundArgs& a = a_;
    if (a.flist_send && !a.fst[kFstBad + (int)(a.g & 1)]) return;   // k_send_list walks this round's list
    extern __shared__ uint64_t s_dyn[];
    uint16_t* s_slots = reinterpret_cast<uint16_t*>(s_dyn);  // [ring] active slots of topic t
    constexpr int kTmChunk = 2 * kTmThreads;                 // peers per chunk (two per thread)
    constexpr int kWv = kTmThreads / 64;
    constexpr uint64_t kChunkWords = (1ull << (kTmChunk / 64)) - 1;
    __shared__ uint32_t s_front[kTmChunk];                   // frontier senders
    __shared__ uint32_t s_from[kTmChunk];                    // their first senders
    __shared__ uint32_t s_off[kTmChunk];                     // first flattened edge of each sender
    __shared__ uint32_t s_beg[kTmChunk];                     // its row's first edge (sedge: first entry)
    __shared__ uint64_t s_msk[kTmChunk];                     // its mesh mask (0: the whole row)
    __shared__ uint8_t s_sk[kTmChunk];                       // its slot (index in the pass)
    __shared__ uint8_t s_pl[kTmChunk];                       // its row's topic slot of t (plane, gsim_internal.h)
    __shared__ uint16_t s_own[kTmWin];                       // sender (index above) of each flattened edge of a window
    // claim-list entries of the iteration's copies
    __shared__ uint64_t s_cl[(SP && !LAT) ? kTmThreads * GSIM_TM_P : 1];
    __shared__ uint32_t s_wsum[64];
    __shared__ uint32_t s_m[kTsSlots], s_org[kTsSlots];      // the pass's slots and their origins
    __shared__ uint64_t s_cb[kTsSlots];                      // ... and their first cells (Cells::cbase)
    __shared__ uint8_t s_vd[kTsSlots], s_ow[kTsSlots], s_wa[kTsSlots], s_lat[kTsSlots];
    __shared__ int s_ns, s_nf;
    __shared__ uint32_t s_ne;
    __shared__ unsigned long long s_clm;                     // slots of the pass with a new claim
    __shared__ unsigned long long s_stats[4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid == 0) { s_stats[0] = s_stats[1] = s_stats[2] = s_stats[3] = 0; }
    unsigned long long n_acc = 0, n_gray = 0, n_first = 0;
#ifdef GSIM_DIAG_PHASE
    TM_CLK(c_start);
    unsigned long long d_scan = 0, d_walk = 0, d_late = 0, n_layers = 0, n_chunks = 0, n_latef = 0;
#endif
    // one (topic, peer range) item per block
    const uint32_t lb = blockIdx.x;
    int32_t t = 0;
    {
        int32_t r = a.T > 0 ? a.T : 1;
        while (r - t > 1) {
            const int32_t mid = (t + r) >> 1;
            if (a.tmtab[mid] <= lb) t = mid; else r = mid;
        }
    }
    const int64_t range = a.tmtab[(a.T > 0 ? a.T : 1) + 1 + t];
    const int64_t pend_ = a.shi;
    const int64_t lo = a.slo + (int64_t)(lb - a.tmtab[t]) * range;
    const int64_t hi = lo + range < pend_ ? lo + range : pend_;
    const int64_t wlo = (int64_t)a.rlo >> 6;
    if (tid == 0) s_ns = 0;
    __syncthreads();
    // a sub-ring (gsim_msg_config.topic_slots) holds topic t's slots alone
    const int m_lo = a.topic_slots > 0 ? t * a.topic_slots : 0;
    const int m_hi = a.topic_slots > 0 ? m_lo + a.topic_slots : a.ring;
    for (int m = m_lo + tid; m < m_hi; m += kTmThreads) {
        if (((a.nnew_prev[m >> 5] >> (m & 31)) & 1u) && (int32_t)a.mtopic[m] == t) {
            const int q = atomicAdd(&s_ns, 1);
            s_slots[q] = (uint16_t)m;
        }
    }
    __syncthreads();
    const int ns = a.g > 0 && lo < pend_ ? s_ns : 0;
    const ctp_t tp = const_tp(a.tp) + t;
    const bool scored_t = tp->scored != 0;
    const int64_t window = tp->mesh_message_deliveries_window_ns;
    const double mcap = tp->mesh_message_deliveries_cap;
    const uint32_t par = (uint32_t)(a.g & 1);
    const uint32_t claim_hi = kClaim | (par << 30);
    for (int k0 = 0; k0 < ns; k0 += kTsSlots) {
        const int nb = ns - k0 < kTsSlots ? ns - k0 : kTsSlots;
        if (tid < nb) {
            const uint32_t m = s_slots[k0 + tid], origin = a.morigin[m];
            s_m[tid] = m;
            s_cb[tid] = a.cs.cbase[m];
            s_org[tid] = origin;
            s_vd[tid] = a.minv[m];
            s_ow[tid] = (origin < a.N && ((a.sub[origin] >> t) & 1ull)) ? GSIM_TF_MESH : GSIM_TF_FANOUT;
            s_wa[tid] = window >= 0 && a.now - round_time(a, a.mpub[m]) <= window;
            if (LAT) s_lat[tid] = a.mlat[m];
        }
        if (tid == 0) s_clm = 0;
        uint64_t clm = 0;
        __syncthreads();
        for (int64_t c0 = lo; c0 < hi; c0 += kTmChunk) {
            TM_CLK(c_chunk);
            // the pass's slots with fresh bits in the chunk: every wave
            // computes the same ballot from the summary words
            const int64_t cw0 = c0 >> 6;
            bool nzs = false;
            if (lane < nb)
                nzs = ((a.fsum[(int64_t)s_m[lane] * a.nsw + (cw0 >> 6)] >> (cw0 & 63)) & kChunkWords) != 0;
            const uint64_t cm = __ballot(nzs);
            if (!cm) continue;                                   // block-uniform
            // thread tid: peers x0, x0 + 1; pm[u] bit k: fresh in the pass's slot k
            const int64_t x0 = c0 + 2 * (int64_t)tid;
            const int64_t wi = x0 >> 6;
            const int sh = (int)(x0 & 63);
            const uint32_t vmask = x0 + 1 < hi ? 3u : 1u;
            uint64_t pm[2] = {0, 0}, nzk = 0;
            if (x0 < hi) {
                uint64_t b = cm;
                while (b) {
                    int kk[4];
                    uint64_t wv[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        kk[q] = b ? __builtin_ctzll(b) : -1;
                        if (b) b &= b - 1;
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) wv[q] = kk[q] >= 0 ? a.fresh[(int64_t)s_m[kk[q]] * a.nw + wi] : 0ull;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (kk[q] < 0) continue;
                        const uint32_t f = (uint32_t)(wv[q] >> sh) & vmask;
                        if (wv[q]) nzk |= 1ull << kk[q];
                        if (f & 1u) pm[0] |= 1ull << kk[q];
                        if (f & 2u) pm[1] |= 1ull << kk[q];
                    }
                }
            }
            bool first_layer = true;
#ifdef GSIM_DIAG_PHASE
            TM_CLK(c_l0);
            TM_ACC(d_scan, c_chunk, c_l0);
#endif
            for (;;) {
                const RoundArgs& a = kernarg0(a_);   // (re-read per layer: SGPR pressure)
                TM_CLK(c_layer);
                const uint32_t fb = (pm[0] ? 1u : 0u) | (pm[1] ? 2u : 0u);
                uint32_t len2[2] = {0, 0}, beg2[2] = {0, 0}, from2[2] = {0, 0}, k2[2] = {0, 0}, pl2[2] = {0, 0};
                uint64_t msk2[2] = {0, 0};
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    if ((fb >> u) & 1u) {
                        k2[u] = (uint32_t)__builtin_ctzll(pm[u]);
                        const uint32_t x = (uint32_t)(x0 + u), m = s_m[k2[u]];
                        // a forwarder's cell (committed)
                        const int64_t xc = SP ? a.cs.at((int64_t)s_cb[k2[u]], t, x) : (int64_t)m * a.cs.n + x;
                        from2[u] = xc >= 0 ? (uint32_t)a.cs.cell[xc] & kPeerMask : kPeerMask;
                        const uint64_t xm = SP ? smask_of(a.smask, x) : ~0ull;
                        pl2[u] = (uint32_t)__popcll(xm & ((1ull << t) - 1ull));
                        const uint32_t rb = a.row_ptr[x], deg = a.row_ptr[x + 1] - rb;
                        if (!slot_has(xm, t)) {
                            // no state for t in x's row (cannot happen: a forwarder holds its
                            // topic, an origin gets the slot at publication): nothing is sent
                        } else if (deg <= 64 && x != s_org[k2[u]]) {
                            msk2[u] = a.mmask[(int64_t)t * a.N + x];
                            beg2[u] = rb;
                            len2[u] = (uint32_t)__popcll(msk2[u]);
                        } else if (a.hlist && x != s_org[k2[u]] &&
                                   a.hlist[((int64_t)a.hidx[x] * a.T + t) * (1 + kHubMesh)] != 0xFFFFFFFFu) {
                            // a hub: its listed mesh | direct edges
                            const uint32_t lo_ = (uint32_t)(((int64_t)a.hidx[x] * a.T + t) * (1 + kHubMesh));
                            beg2[u] = kHubList | (lo_ + 1u);
                            len2[u] = a.hlist[lo_];
                        } else {
                            const uint32_t* rp = a.sptr ? a.sptr : a.row_ptr;
                            beg2[u] = rp[x];
                            len2[u] = rp[x + 1] - beg2[u];
                        }
                    }
                }
                uint32_t vc = (uint32_t)__popc(fb), ve = len2[0] + len2[1];
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t yc = (uint32_t)__shfl_up((int)vc, o, 64), ye = (uint32_t)__shfl_up((int)ve, o, 64);
                    if (lane >= o) { vc += yc; ve += ye; }
                }
                if (lane == 63) { s_wsum[wid] = vc; s_wsum[16 + wid] = ve; }
                __syncthreads();
                if (tid < 64) {
                    const uint32_t c = tid < kWv ? s_wsum[tid] : 0u, e = tid < kWv ? s_wsum[16 + tid] : 0u;
                    uint32_t ic = c, ie = e;
                    for (int o = 1; o < kWv; o <<= 1) {
                        const uint32_t yc = (uint32_t)__shfl_up((int)ic, o, 64), ye = (uint32_t)__shfl_up((int)ie, o, 64);
                        if (lane >= o) { ic += yc; ie += ye; }
                    }
                    if (tid < kWv) { s_wsum[32 + tid] = ic - c; s_wsum[48 + tid] = ie - e; }
                    if (tid == kWv - 1) { s_nf = (int)ic; s_ne = ie; }
                }
                __syncthreads();
                {
                    uint32_t q = s_wsum[32 + wid] + vc - (uint32_t)__popc(fb);
                    uint32_t off = s_wsum[48 + wid] + ve - (len2[0] + len2[1]);
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        if ((fb >> u) & 1u) {
                            s_front[q] = (uint32_t)(x0 + u);
                            s_from[q] = from2[u];
                            s_off[q] = off;
                            s_beg[q] = beg2[u];
                            s_msk[q] = msk2[u];
                            s_sk[q] = (uint8_t)k2[u];
                            s_pl[q] = (uint8_t)pl2[u];
                            ++q;
                            off += len2[u];
                        }
                    }
                    if (first_layer) {
                        // the bits are read: clear them (one thread per word)
                        if ((x0 & 63) == 0)
                            for (uint64_t b = nzk; b; b &= b - 1)
                                a.fresh[(int64_t)s_m[__builtin_ctzll(b)] * a.nw + wi] = 0;
                        if (tid < nb && ((cm >> tid) & 1ull))
                            atomicAnd(reinterpret_cast<unsigned long long*>(a.fsum + (int64_t)s_m[tid] * a.nsw + (cw0 >> 6)),
                                      ~(kChunkWords << (cw0 & 63)));
                    }
                }
                __syncthreads();
                const int nf = s_nf;
                const uint32_t ne = s_ne;
#ifdef GSIM_DIAG_PHASE
                TM_CLK(c_walk);
                TM_ACC(d_scan, c_layer, c_walk);
                if (!first_layer) TM_ACC(d_late, c_layer, c_walk);
                n_layers++;
                if (first_layer) n_chunks++;
                else n_latef += (unsigned long long)s_nf;
#endif
                if (nf > 0) {
                    constexpr int P = GSIM_TM_P;
                    constexpr uint32_t kPerIt = kTmThreads * P;
                    static_assert(kTmWin % kPerIt == 0, "whole iterations per window");
                  // dense chunks table each flattened edge's sender in LDS (written by
                  // the senders); sparse ones search the offsets per edge
                  const bool tab = nf >= kTmTabMin;
                  for (uint32_t w0 = 0; w0 < ne; w0 += tab ? kTmWin : ne) {
                    const uint32_t w1 = (!tab || ne - w0 < kTmWin) ? ne : w0 + kTmWin;
                    if (tab) {
                        for (int q = tid; q < nf; q += kTmThreads) {
                            const uint32_t o0 = s_off[q], o1 = q + 1 < nf ? s_off[q + 1] : ne;
                            const uint32_t lo_f = o0 > w0 ? o0 : w0, hi_f = o1 < w1 ? o1 : w1;
                            for (uint32_t f = lo_f; f < hi_f; ++f) s_own[f - w0] = (uint16_t)q;
                        }
                        __syncthreads();
                    }
                    for (uint32_t it0 = w0; it0 < w1; it0 += kPerIt) {
                        const RoundArgs& a = kernarg0(a_);   // (re-read per iteration: SGPR pressure)
                        uint32_t jv[P], fv[P], ev[P], iv[P], nv[P], kv[P];
                        int64_t pv[P];           // the sender's plane of topic t
                        uint8_t mfv[P], dsv[P], tfv[P];
                        bool vv[P], mk[P];
                        double xv[P];
#pragma unroll
                        for (int u = 0; u < P; ++u) {
                            const uint32_t fi = it0 + (uint32_t)(u * kTmThreads + tid);
                            vv[u] = fi < w1;
                            int q = 0;
                            if (vv[u] && tab) {
                                q = (int)s_own[fi - w0];
                            } else if (vv[u]) {
                                int l = 0, r = nf;
                                while (r - l > 1) {
                                    const int mid = (l + r) >> 1;
                                    if (s_off[mid] <= fi) l = mid; else r = mid;
                                }
                                q = l;
                            }
                            jv[u] = vv[u] ? s_front[q] : 0u;
                            fv[u] = vv[u] ? s_from[q] : 0u;
                            kv[u] = vv[u] ? s_sk[q] : 0u;
                            pv[u] = !vv[u] ? 0 : (SP && a.smask) ? (int64_t)s_pl[q] * a.E : (int64_t)t * a.E;
                            const uint32_t k = fi - s_off[q];
                            const uint64_t msk = s_msk[q];
                            const uint32_t bq = s_beg[q];
                            mk[u] = msk != 0 || (bq & kHubList);
                            if (msk) ev[u] = bq + kth_bit(msk, k);
                            else if (bq & kHubList) ev[u] = vv[u] ? a.hlist[(bq & ~kHubList) + k] : 0u;
                            else if (a.sedge && vv[u]) ev[u] = a.sedge[bq + k];
                            else ev[u] = s_beg[q] + k;
                        }
                        uint32_t xq[PUSH ? P : 1];   // PUSH: the copy's bit (a cross edge), ~0: an owned receiver
                        uint64_t xbk[PUSH ? P : 1];  // ... a remote copy's xbits word (~0: none) and bit
                        uint64_t xbv[PUSH ? P : 1];
#pragma unroll
                        for (int u = 0; u < P; ++u) {
                            iv[u] = 0; mfv[u] = 0; dsv[u] = 0; tfv[u] = 0; nv[u] = 0; xv[u] = 0.0;
                            if constexpr (PUSH) { xq[u] = ~0u; xbk[u] = ~0ull; xbv[u] = 0; }
                            if (vv[u]) {
                                const uint32_t e = ev[u];
                                const uint8_t vd = s_vd[kv[u]];
                                // a masked row's positions are its mesh (or direct) edges: the
                                // router flags are read only for direct ones (below)
                                const int64_t pe = pv[u] + e;
                                iv[u] = a.col[e]; dsv[u] = a.dstate[e];
                                if (!mk[u]) mfv[u] = a.mflags[pe];
                                if constexpr (PUSH) {
                                    xq[u] = a.xwq[e];
                                } else {
                                    tfv[u] = a.tflags[pe];
                                    if (verdict_penalises(vd)) xv[u] = a.invalid[pe];
                                    else if (vd == GSIM_VERDICT_ACCEPT) nv[u] = a.mcnt[pe];
                                }
                            }
                        }
                        if constexpr (PUSH) {
                            // the records of owned receivers only: a ghost's shard holds its own
#pragma unroll
                            for (int u = 0; u < P; ++u) {
                                if (vv[u] && xq[u] == ~0u) {
                                    const uint8_t vd = s_vd[kv[u]];
                                    const int64_t pe = pv[u] + ev[u];
                                    tfv[u] = a.tflags[pe];
                                    if (verdict_penalises(vd)) xv[u] = a.invalid[pe];
                                    else if (vd == GSIM_VERDICT_ACCEPT) nv[u] = a.mcnt[pe];
                                }
                            }
                        }
                        int qpl[P];              // validation latency: queue plane of the copy (-1: none)
                        uint64_t qv[P];
                        uint32_t clw = 0;        // bit u: copy u claimed an unseen cell (its entry in s_cl)
#pragma unroll
                        for (int u = 0; u < P; ++u) { qpl[u] = -1; qv[u] = 0; }
#pragma unroll
                        for (int u = 0; u < P; ++u) {
                            const uint32_t j = jv[u], e = ev[u], i = iv[u], k = kv[u];
                            const uint32_t m = s_m[k], origin = s_org[k];
                            const uint8_t vd = s_vd[k];
                            const bool inv = vd != GSIM_VERDICT_ACCEPT;
                            const bool pen = verdict_penalises(vd), seeable = vd != GSIM_VERDICT_SIGNATURE;
                            const uint8_t ds = dsv[u], tf = tfv[u];
                            bool sel;
                            if (mk[u]) sel = !(ds & GSIM_DS_DIRECT) || (a.mflags[pv[u] + e] & GSIM_TF_MESH);
                            else sel = (mfv[u] & (j == origin ? s_ow[k] : GSIM_TF_MESH)) != 0;
                            if (a.flood && vv[u] && j == origin)
                                sel = ((a.sub[i] >> t) & 1ull) &&
                                      ((a.sharded && (j < a.rlo || j >= a.rhi)) ? a.pgate[e] != 0
                                                                                : a.score[a.rev[e]] >= a.pub_thr);
                            if (vv[u] && (ds & GSIM_DS_DIRECT) && !sel) sel = (a.sub[i] >> t) & 1ull;
                            const bool tg = vv[u] && sel && (ds & GSIM_DS_CONNECTED) && i != fv[u] && i != origin;
                            const bool remote = i < a.rlo || i >= a.rhi;
                            if (tg && a.tr.ev) {         // the copy's RPC: SendRPC / RecvRPC (trace.go:250-297)
                                const int64_t ts = round_time(a, a.g);
                                const uint64_t tm = ((uint64_t)a.g << 32) | m;
                                if (a.tr.on(j)) a.tr.push(ts, tm, j, i, t, GSIM_TRACE_SEND_RPC, 0);
                                // (a pushed copy's RecvRPC: only the sender's shard knows of it)
                                if (a.tr.on_any(i)) a.tr.push(ts, tm, i, j, t, GSIM_TRACE_RECV_RPC, 0);
                            }
                            if constexpr (PUSH) {
                                // the receiver's shard delivers it (its AcceptFrom, records, cell):
                                // its bit, set below for the whole wave (xbits_or_wave)
                                if (tg && remote) {
                                    const uint32_t xb = xq[u];
                                    xbk[u] = (uint64_t)((int64_t)m * a.xbw + (xb >> 6));
                                    xbv[u] = 1ull << (xb & 63u);
                                    continue;
                                }
                            }
                            const bool ok = tg && !remote && (ds & GSIM_DS_ACCEPT);
                            n_gray += tg && !remote && !ok;
                            if (!ok) continue;
                            if constexpr (GT) {                  // the peer gater (gater_accept)
                                if (!gater_accept(a, i, e, m, j)) continue;
                            }
                            // a topic the receiver left: skipped (pubsub.go:1094-1098)
                            if (a.subdyn && !((a.sub[i] >> t) & 1ull)) continue;
                            if constexpr (GT) gater_copy(a, e, !seeable);
                            n_acc++;
                            if (a.tr.on(i))
                                a.tr.push(round_time(a, a.g), ((uint64_t)a.g << 32) | m, i, j, t,
                                          seeable ? kTraceCopy : (uint8_t)GSIM_TRACE_REJECT_MESSAGE, vd);
                            const bool sc = scored_t && (ds & GSIM_DS_TRACKED);
                            const uint32_t L = LAT ? s_lat[k] : 0u;
                            const uint64_t* s_bm = a.seenbm + (int64_t)m * a.nw + wlo;
                            const int64_t bw = ((int64_t)i >> 6) - wlo;
                            // a committed cell need not be read when the copy cannot be
                            // credited; with a validation latency the credit is decided at
                            // completion (mesh and record then), so only an unscored topic
                            // or an ignored / throttled message skips it
                            const bool sbit = (s_bm[bw] >> (i & 63)) & 1ull;   // committed before this round
                            const bool known = sbit && (L ? (!scored_t || (inv && !pen))
                                                          : (s_wa[k] || !sc || inv || !(tf & GSIM_TF_IN_MESH)));
                            // the receiver's cell (a member of t: mesh, direct, fanout and flood
                            // targets all hold the topic, §2); -1 cannot happen
                            const int64_t ci = known ? 0 : SP ? a.cs.at((int64_t)s_cb[k], t, i) : (int64_t)m * a.cs.n + i;
                            if (SP && ci < 0) continue;
                            uint32_t lo_w = j;
                            if (sc && !inv) {
                                lo_w |= kCreditFirst;
                                if (window < 0 && (tf & GSIM_TF_IN_MESH)) lo_w |= kCreditMesh;
                            }
                            const uint64_t cv = ((uint64_t)(claim_hi | e) << 32) | lo_w;
                            // a receiver that had not seen m before this round (no claims of
                            // round g-1 remain without a latency): the claim is the cell's only
                            // access -- atomicMin keeps a lower edge's claim of this round and
                            // returns what the cell held (a load, then the claim, otherwise)
                            const bool fold = !LAT && !sbit && seeable;
#if defined(GSIM_DIAG_CLAIM)
                            // timing diagnostic (wrong first-delivery totals; 2: racy winners)
                            uint64_t c;
                            if (known) c = 0ull;
                            else if (fold) {
#if GSIM_DIAG_CLAIM == 1
                                __hip_atomic_fetch_min(a.cs.cell + ci, cv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
                                a.cs.cell[ci] = cv;
#endif
                                c = kUnseen64;
                            } else c = a.cs.cell[ci];
#else
                            const uint64_t c = known ? 0ull
                                             : fold ? __hip_atomic_fetch_min(a.cs.cell + ci, cv, __ATOMIC_RELAXED,
                                                                             __HIP_MEMORY_SCOPE_AGENT)
                                                    : a.cs.cell[ci];
#endif
                            const uint32_t chi = (uint32_t)(c >> 32);
                            // the round validation completed (or completes) in; -1: unclaimed
                            // or claimed in this round
                            int64_t seen_round = -1;
                            if (known) seen_round = a.g - 1;
                            else if (c != kUnseen64) {
                                if (!(chi & kClaim)) seen_round = chi;
                                else if (((chi >> 30) & 1u) != par) seen_round = a.g - 1 + L;
                            }
                            if (fold || (seeable && seen_round < 0 && (c == kUnseen64 || (chi & kEdgeMask) > e))) {
                                const uint64_t prev = fold ? c
                                                           : __hip_atomic_fetch_min(a.cs.cell + ci, cv, __ATOMIC_RELAXED,
                                                                                    __HIP_MEMORY_SCOPE_AGENT);
                                if (prev == kUnseen64) {
                                    n_first++;
                                    clm |= 1ull << k;
                                    if constexpr (SP && !LAT) {
                                        clw |= 1u << u;
                                        s_cl[u * kTmThreads + tid] = cl_entry(a, i, m, ci, (int64_t)s_cb[k]);
                                    }
                                }
                            }
                            if (L && seeable && (seen_round < 0 || seen_round > a.g)) {
                                // the receiver is still validating: drec.peers (score.go:806-809)
                                if (scored_t && (pen || !inv)) {
                                    const int pl = (int)((seen_round < 0 ? a.g + L : seen_round) & (kVqPlanes - 1));
                                    // dense layout: a count on the record (this block's alone,
                                    // as mcnt), else / when full a queue entry
                                    bool counted = false;
                                    if (a.vpc) {
                                        uint8_t* cp = a.vpc + ((int64_t)(pen ? kVqPlanes : 0) + pl) * a.vpe + pv[u] + e;
                                        const uint8_t x = *cp;
                                        if (x < 255u) { *cp = (uint8_t)(x + 1u); counted = true; }
                                    }
                                    if (!counted) {
                                        qpl[u] = pl;
                                        qv[u] = vq_entry(e, t, pen ? kVqInv : kVqDup);
                                    }
                                }
                                continue;
                            }
                            if (!sc) continue;
                            const int64_t ir = pv[u] + e;
                            if (pen) {
                                a.invalid[ir] = xv[u] + 1.0;
                                inv_mark(a);
                            } else if (!inv && (tf & GSIM_TF_IN_MESH)) {
                                const bool in_window = known ? true
                                                     : seen_round >= 0 ? (a.now - round_time(a, seen_round) <= window)
                                                                       : (window >= 0);
                                if (in_window) {
                                    uint32_t n = nv[u];
                                    if (n == 255u) {
                                        a.meshd[ir] = apply_incs(a.meshd[ir], n, mcap);
                                        n = 0;
                                    }
                                    a.mcnt[ir] = (uint8_t)(n + 1);
                                }
                            }
                        }
                        if constexpr (PUSH) {
#pragma unroll
                            for (int u = 0; u < P; ++u) xbits_or_wave(a.xbits, xbk[u], xbv[u]);
                        }
                        if constexpr (LAT) {
#pragma unroll
                            for (int u = 0; u < P; ++u) vq_push_wave(a, qpl[u], qv[u]);
                        }
                        if constexpr (SP && !LAT) {
                            if (a.clist) {
#pragma unroll
                                for (int u = 0; u < P; ++u)
                                    clist_push_wave(a, (clw >> u) & 1u, s_cl[u * kTmThreads + tid]);
                            }
                        }
                    }
                    if (tab) __syncthreads();                    // s_own is rewritten by the next window
                  }
                }
#ifdef GSIM_DIAG_PHASE
                {
                    TM_CLK(c_wend);
                    TM_ACC(d_walk, c_walk, c_wend);
                    if (!first_layer) TM_ACC(d_late, c_walk, c_wend);
                }
#endif
                // the next layer: each peer's next slot
                first_layer = false;
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    if (pm[u]) pm[u] &= pm[u] - 1;
                if (!__syncthreads_or((pm[0] | pm[1]) != 0)) break;   // also: s_front is rewritten next
            }
        }
        // slots that stay active next round: a copy claimed a new cell
        if (clm) atomicOr(&s_clm, (unsigned long long)clm);
        __syncthreads();
        if (tid < nb && ((s_clm >> tid) & 1ull)) {
            const uint32_t m = s_m[tid];
            slots_claimed(a, (int)(m >> 5), 1u << (m & 31));
        }
        __syncthreads();                                         // the pass's slot table is rewritten next
    }
    n_acc = wave_sum_u64(n_acc);
    n_gray = wave_sum_u64(n_gray);
    n_first = wave_sum_u64(n_first);
    if (lane == 0 && (n_acc | n_gray)) {
        atomicAdd(&s_stats[0], n_acc);
        atomicAdd(&s_stats[1], n_first);
        atomicAdd(&s_stats[3], n_gray);
    }
    __syncthreads();
    if (tid == 0 && (s_stats[0] | s_stats[3])) {
        stats_add(a, s_stats[0], s_stats[1], s_stats[3]);
    }
#ifdef GSIM_DIAG_PHASE
    TM_CLK(c_end);
    if (lane == 0) {
        atomicAdd(&g_tm_diag[0], c_end - c_start);
        atomicAdd(&g_tm_diag[1], d_scan);
        atomicAdd(&g_tm_diag[2], d_walk);
        atomicAdd(&g_tm_diag[3], 1ull);
        atomicAdd(&g_tm_diag[4], d_late);
        if (tid == 0) {
            atomicAdd(&g_tm_diag[5], n_layers);
            atomicAdd(&g_tm_diag[6], n_chunks);
            atomicAdd(&g_tm_diag[7], n_latef);
        }
    }
#endif
}

// Commit every claim of round g (markSeen + P2 credit) before the state is
// read or changed by anything but the next round.
// SPLIT (a shard's few words: a wave per word leaves the CUs idle): the slots
// shared over gridDim.y groups by topic, so the record credits and lastput
// stay plain stores (two slots of one topic can credit the same record)
template <bool LAT, bool SP, bool GT = false, bool SPLIT = false>
__global__ __launch_bounds__(256) void k_commit(RoundArgs a)
{
    extern __shared__ uint16_t s_act[];
    __shared__ int s_n;
    if (a.clist && !a.clist_n[kClSub * kClStride]) return;   // the claim list covers the round (k_commit_list)
    // this scan sets the fresh bits: round g+1's forwarder list is incomplete
    if (a.flist && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) a.fst[kFstBad + (int)((a.g + 1) & 1)] = 1;
    // SPLIT: group y takes the slots of topics t = y mod gridDim.y, whose
    // credits no other group can touch -- plain stores (serial K = 8 C3 mean
    // shard 11.53 / 11.55 against 11.61 / 11.63 ms with the slot batches dealt
    // over the groups and atomic credits, gpurun_out/r05p_ab)
    const int nact = SPLIT ? active_slots_topics(a.nnew_cur, a.ring, a.mtopic, (int)blockIdx.y, (int)gridDim.y,
                                                       s_act, &s_n)
                                 : active_slots(a.nnew_cur, a.ring, s_act, &s_n);
    const int lane = threadIdx.x & 63;
    // claims exist only at receivers' cells: the words of [rlo, rhi), a wave per
    // word, grid-stride (a launch that exits early stays cheap: c5's 39k blocks
    // cost 1 ms per round doing nothing)
    for (int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);; wv += (int64_t)gridDim.x * 4) {
        const int64_t i0 = ((int64_t)a.rlo & ~63ll) + wv * 64;
        if (i0 >= (int64_t)a.rhi || nact == 0) return;
        const int64_t i = i0 + lane;
        const bool vi = i < a.CN;
        const uint32_t par = (uint32_t)(a.g & 1);
        // (SPLIT: the group's slots in batches of kSplitBatch -- parallel waves
        // over the groups instead of cells in flight per wave)
        constexpr int kB = SPLIT ? kSplitBatch : kSlotBatch;
        for (int k0 = 0; k0 < nact; k0 += kB) {
            uint64_t cv[kB];
            int64_t ci[SP ? kB : 1];           // the dense layout recomputes m * N + i
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const int k = k0 + b;
                const int64_t c = (k < nact && vi) ? word_cell<SP>(a.cs, a.mtopic, s_act[k], i0 >> 6, lane) : -1;
                if constexpr (SP) ci[b] = c;
                cv[b] = c >= 0 ? a.cs.cell[c] : kUnseen64;
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const int k = k0 + b;
                const uint64_t cb = __ballot(k < nact && is_claim_of(cv[b], par));
                if (cb && lane == 0) {
                    const uint32_t m = s_act[k];
                    a.seenbm[(int64_t)m * a.nw + (i0 >> 6)] |= cb;
                    // receivers forward what they accepted, in the next round
                    if (a.fresh && a.minv[m] == GSIM_VERDICT_ACCEPT && (!LAT || !a.mlat[m])) {
                        // fire-and-forget atomics: the wave does not wait on them
                        atomicOr(reinterpret_cast<unsigned long long*>(a.fresh + (int64_t)m * a.nw + (i0 >> 6)), cb);
                        atomicOr(reinterpret_cast<unsigned long long*>(a.fsum + (int64_t)m * a.nsw + (i0 >> 12)),
                                 1ull << ((i0 >> 6) & 63));
                    }
                }
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const int k = k0 + b;
                if (k >= nact) break;
                int qpl = -1;
                uint64_t qv = 0;
                if (is_claim_of(cv[b], par)) {
                    const uint32_t m = s_act[k];
                    uint64_t* cp = a.cs.cell + (SP ? ci[b] : (int64_t)m * a.cs.n + i);
                    commit_claim<false, LAT, SP, GT>(a, cp, cv[b], a.g, m, i, &qpl, &qv);
                }
                if constexpr (LAT) vq_push_wave(a, qpl, qv);
            }
        }
        if constexpr (!SP && !SPLIT) return;              // dense: a launch covers every word
    }
}

// The same commits from the claim list (member-compacted cells: a round's
// claims are few next to its active slots x peers): one thread per claimed
// cell; several claims may share a bitmap word, a lastput or a winner's
// record, so those updates are atomic.  An overflowed list leaves the round
// to k_commit's word scan.
template <bool SP>
__global__ __launch_bounds__(256) void k_commit_list(RoundArgs a)
{
    if (a.clist_n[kClSub * kClStride]) return;
    const uint32_t q = blockIdx.y;                       // sub-list
    const int64_t n = (int64_t)a.clist_n[q * kClStride];
    const uint32_t par = (uint32_t)(a.g & 1);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // (grid-stride with a wave-uniform trip count: flist_push_wave is called by every lane)
    for (int64_t k0 = (int64_t)blockIdx.x * blockDim.x; k0 < n; k0 += stride) {
        const int64_t k = k0 + threadIdx.x;
        bool fw = false;
        uint64_t fv = 0;
        if (k < n) {
            const uint64_t v = a.clist[(int64_t)q * a.clist_cap + k];
            const uint32_t i = a.cl_j ? (uint32_t)(v & (kClPeerMax - 1)) : (uint32_t)v;
            const uint32_t m = a.cl_j ? (uint32_t)((v >> 24) & 0x1FFFu) : (uint32_t)(v >> 32);
            const int64_t ci = a.cl_j ? (int64_t)a.cs.cbase[m] + (int64_t)(v >> 37)
                             : SP ? a.cs.idx(m, (int32_t)a.mtopic[m], i) : (int64_t)m * a.cs.n + i;
            uint64_t* cp = ci >= 0 ? a.cs.cell + ci : nullptr;
            const uint64_t c = cp ? *cp : kUnseen64;
            if (cp && is_claim_of(c, par)) {
                const int64_t w = (int64_t)(i >> 6);
                const uint64_t bit = 1ull << (i & 63);
                atomicOr(reinterpret_cast<unsigned long long*>(a.seenbm + (int64_t)m * a.nw + w), bit);
                if (a.fresh && a.minv[m] == GSIM_VERDICT_ACCEPT) {
                    if (a.flist_commit) { fw = true; fv = fl_entry(a, i, m, (uint32_t)c & kPeerMask); }   // round g+1's list
                    // (a shard's holder accumulation reads the fresh bits before the send)
                    if (!a.flist_commit || a.sharded) fresh_set(a, m, w, bit);
                }
                if (a.gt.act) commit_claim<true, false, SP, true>(a, cp, c, a.g, m, i);
                else commit_claim<true, false, SP>(a, cp, c, a.g, m, i);
            }
        }
        if (a.flist_commit) flist_push_wave(a, a.g + 1, fw, fv);
    }
}

// ---------------------------------------------------------------------------
// Gossip.  Heartbeat k's emitGossip marked ihave[t][e] in
// the receivers' rows (heartbeat.hip).  Control round 0 of tick k runs
// handleIHave for every receiver, and — because nothing a handleIWant gate
// reads can change between rounds 0 and 1 (score snapshot, mcache window,
// behaviour) — the advertisers' handleIWant with it: the messages they send
// are queued for round 2.  A receiver gets one IHAVE RPC per advertiser per
// heartbeat, so handleIHave sees peerhave = 1 and iasked = 0
// (gossipsub.go:638-648).  The MaxIHaveLength truncations (emitGossip's
// per-peer subset, gossipsub.go:1763-1772; the IWANT cap, 679-690) can only
// apply when the window holds more than MaxIHaveLength slots: then
// k_ihave_pairs runs instead of k_ihave.  mcache.peertx (GetForPeer's count,
// mcache.go:73-86) can exceed 1 only for a message its receiver never marks
// seen — a bad signature, served by its origin alone — and is counted per
// (slot, origin's row position) for those (Deliver::d_peertx).

struct IhArgs {
    int64_t N, E;
    int32_t T, ring, R;
    int64_t g, tick;
    int32_t lo_round;              // first round of the gossip window
    const uint32_t *row_ptr, *col, *rev;
    const uint64_t* sub;
    const uint64_t* smask;         // topic slots (gsel planes: the advertiser's row)
    const uint32_t *mtopic, *morigin;
    const uint8_t* minv;
    const uint8_t* mlat;           // validation latencies (RoundArgs::mlat)
    Cells cs;                      // the seen-set (gsim_internal.h)
    const int32_t* slot_last;
    const uint8_t *gsel, *gstate, *behaviour;
    uint64_t* pcand;
    uint32_t* prom;
    int32_t P, prom_idx;
    uint64_t* resp;
    uint32_t* nresp;               // [0] count, [1] overflow
    int64_t resp_cap;
    unsigned long long* gstats;    // [0] receivers x slots walked, [1] IWANT ids, [2] responses, [3] broken promises
    bool respond;                  // GossipRetransmission >= 1
    uint64_t seed;
    int64_t CN;                    // local peers (RoundArgs)
    // sharded network: receivers are the owned peers [rlo, rhi) and every slot
    // is pulled (receivers walk); a ghost advertiser's holding is its ghost
    // cell (first-seen rounds its shard exported); keys use global ids
    uint32_t rlo, rhi;
    int32_t sharded;
    const uint32_t* gid;
    int32_t max_ihave;             // MaxIHaveLength
    // GetForPeer counts of bad-signature slots: [ring][ptx_w] by the origin's row position
    uint8_t* peertx;
    int32_t ptx_w;
    int32_t retrans;               // GossipRetransmission
    // member-major walk (Deliver::d_mlist): blocks of a topic's members
    const uint32_t* mlist;
    const int64_t *mloff, *mcount;
    const uint32_t* mmtab;
    int32_t topic_slots;
    // MM on sub-rings of at most 128 slots (Deliver::d_ihm): per member, the window slots
    // held and unseen, written by k_gossip_count_mm, read by k_ihave instead of the cells
    uint64_t* ihm;
    const int64_t* mmb;
    // MM hub rows (k_ihave LP 1 / 2): the listed waves (block * 4 + wave) and their count
    uint32_t* hubw;
    uint32_t* hubn;
    // trace: the IWANT requests' RPCs (round times as RoundArgs)
    TraceRef tr;
    int64_t t0, hb;
    const int64_t* roff;
};

// The IWANT of receiver p to advertiser i (handleIHave's reply, HandleRPC ->
// sendRPC, gossipsub.go:611-627, 1195-1200) asks for message slot m: one
// record per id of the RPC (reason 2; gsim_trace_encode joins a request's ids
// into one ControlMeta.iwant), SendRPC at p in control round g and RecvRPC at i
// in round g + 1, where handleIWant runs.
__device__ __forceinline__ void trace_iwant(const IhArgs& a, uint32_t p, uint32_t i, uint32_t m)
{
    auto rt = [&](int64_t g) {
        const uint32_t q = (uint32_t)g / (uint32_t)a.R;
        return a.t0 + (int64_t)q * a.hb + a.roff[(uint32_t)g - q * (uint32_t)a.R];
    };
    const uint64_t tm = ((uint64_t)a.g << 32) | m;
    const int32_t t = (int32_t)a.mtopic[m];
    if (a.tr.on(p)) a.tr.push(rt(a.g), tm, p, i, t, GSIM_TRACE_SEND_RPC, 2);
    if (a.tr.on_any(i)) a.tr.push(rt(a.g + 1), tm, i, p, t, GSIM_TRACE_RECV_RPC, 2);
}

// Member-major blocks: block b of a launch over topics' member ranges (table
// tab[T+1] of first blocks) -> its topic.
__device__ __forceinline__ int32_t block_topic(const uint32_t* tab, int32_t T, uint32_t b)
{
    int32_t t = 0, r = T > 0 ? T : 1;
    while (r - t > 1) {
        const int32_t mid = (t + r) >> 1;
        if (tab[mid] <= b) t = mid; else r = mid;
    }
    return t;
}
__device__ __forceinline__ uint32_t member_peer(const IhArgs& a, int32_t t, int64_t j)
{
    const int64_t off = a.mloff[t];
    return off < 0 ? (uint32_t)j : a.mlist[off + j];
}

// handleIWant's GetForPeer count (mcache.go:73-86) for a response to
// (slot m, the advertiser's edge re): only a bad-signature message can be
// asked for twice (its receivers never see it), and only its origin serves it.
__device__ __forceinline__ bool peertx_allows(const IhArgs& a, uint32_t m, uint32_t re, uint32_t advertiser)
{
    if (a.minv[m] != GSIM_VERDICT_SIGNATURE || !a.peertx) return true;
    uint8_t* c = a.peertx + (int64_t)m * a.ptx_w + (re - a.row_ptr[advertiser]);
    const uint32_t n = (uint32_t)*c + 1u;
    *c = (uint8_t)(n > 255u ? 255u : n);
    return (int32_t)n <= a.retrans;
}

// round a cell's message was (or will be) validated and put in the mcache,
// at control time of round g (any claim still pending is from round g-1 or
// g and completes L rounds later), or -1
__device__ __forceinline__ int64_t cell_round(uint64_t c, int64_t g, uint32_t L = 0)
{
    if (c == kUnseen64) return -1;
    const uint32_t hi = (uint32_t)(c >> 32);
    if (!(hi & kClaim)) return hi;
    return ((((hi >> 30) & 1u) == (uint32_t)(g & 1)) ? g : g - 1) + L;
}

constexpr int kRespStage = 256;    // per-wave LDS staging of queued responses

// Direction choice per slot (as in direction-optimizing BFS): a message few
// peers hold is handled from its holders (each walks its row for the peers it
// gossiped to: "push"); one few peers still miss, from those receivers (each
// walks its row for advertisers: "pull").  Both enumerate exactly the same
// (receiver, advertiser, message) IWANT triples.
__device__ __forceinline__ bool holds_in_window(uint64_t c, int64_t g, int32_t lo_round, int64_t tick_round,
                                                bool inv, bool is_origin, uint32_t L)
{
    const int64_t fr = cell_round(c, g, L);
    return fr >= lo_round && fr < tick_round && (!inv || is_origin);
}

template <bool LAT, bool SP>
__global__ __launch_bounds__(256) void k_gossip_count(IhArgs a, uint32_t* gcount)
{
    extern __shared__ uint16_t s_act[];   // [ring] candidate slots, then [2][ring] u32 counters
    __shared__ int s_n;
    uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_act + ((a.ring + 1) & ~1));
    for (int w = threadIdx.x; w < 2 * a.ring; w += blockDim.x) s_cnt[w] = 0;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        int n = 0;
        for (int m0 = 0; m0 < a.ring; m0 += 64) {
            const int m = m0 + lane;
            const bool act = m < a.ring && a.slot_last[m] >= a.lo_round;
            const uint64_t b = __ballot(act);
            if (act) s_act[n + __popcll(b & ((1ull << lane) - 1))] = (uint16_t)m;
            n += __popcll(b);
        }
        if (lane == 0) s_n = n;
    }
    __syncthreads();
    // more slots in the gossip window than MaxIHaveLength: a truncation may
    // apply, k_ihave_pairs handles this stage (bit 2)
    if (blockIdx.x == 0 && threadIdx.x == 0 && s_n > a.max_ihave) atomicOr(&a.nresp[3], 4u);
    const int lane = threadIdx.x & 63;
    const int64_t p0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;   // peers p0 .. p0 + 63
    const int nact = p0 < a.CN ? s_n : 0;
    const int64_t pc = p0 + lane, pl = pc;
    const bool vp = pc < a.CN;
    const uint64_t subp = vp ? a.sub[pl] : 0ull;
    const int64_t tick_round = a.tick * a.R;
    for (int k0 = 0; k0 < nact; k0 += kSlotBatch) {
        uint64_t cv[kSlotBatch];
#pragma unroll
        for (int b = 0; b < kSlotBatch; ++b) {
            const int k = k0 + b;
            // a peer without a cell (not a member of the slot's topic) has not seen it
            const int64_t ci = (k < nact && vp) ? word_cell<SP>(a.cs, a.mtopic, s_act[k], p0 >> 6, lane) : -1;
            cv[b] = ci >= 0 ? a.cs.cell[ci] : kUnseen64;
        }
#pragma unroll
        for (int b = 0; b < kSlotBatch; ++b) {
            const int k = k0 + b;
            if (k >= nact) break;
            const uint32_t m = s_act[k];
            const int32_t t = (int32_t)a.mtopic[m];
            const bool hold = vp && holds_in_window(cv[b], a.g, a.lo_round, tick_round, a.minv[m] != 0,
                                                   (uint32_t)pl == a.morigin[m], LAT ? a.mlat[m] : 0u);
            const bool want = vp && cv[b] == kUnseen64 && ((subp >> t) & 1ull) && pl >= a.rlo && pl < a.rhi;
            const int nh = __popcll(__ballot(hold)), nw = __popcll(__ballot(want));
            if (lane == 0 && nh) atomicAdd(&s_cnt[m], (uint32_t)nh);
            if (lane == 0 && nw) atomicAdd(&s_cnt[a.ring + m], (uint32_t)nw);
        }
    }
    __syncthreads();
    for (int w = threadIdx.x; w < 2 * a.ring; w += blockDim.x)
        if (s_cnt[w]) atomicAdd(&gcount[w], s_cnt[w]);
}

// k_gossip_count over the members of each topic (sub-rings with
// member-compacted cells): block b takes 1024 members of its topic, whose
// cells in each of the topic's slots are consecutive; only the topic's own
// sub-ring is scanned.  Counts are the same as k_gossip_count's: a peer
// without a cell neither holds nor wants.
#ifndef GSIM_COUNT_BATCH
#define GSIM_COUNT_BATCH 4
#endif
constexpr int kCountBatch = GSIM_COUNT_BATCH;    // window slots whose cells one lane loads at once
template <bool LAT>
__global__ __launch_bounds__(256) void k_gossip_count_mm(IhArgs a, const uint32_t* mctab, uint32_t* gcount)
{
    extern __shared__ uint32_t s_c[];     // [2][R] holders, wanting receivers per slot of the sub-ring
    __shared__ uint16_t s_slot[kMaxRing / 8];
    __shared__ int s_n;
    const int32_t t = block_topic(mctab, a.T, blockIdx.x);
    const int32_t R = a.topic_slots, m_lo = t * R;
    for (int w = threadIdx.x; w < 2 * R; w += blockDim.x) s_c[w] = 0;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x < 64) {
        int n = 0;
        for (int k0 = 0; k0 < R; k0 += 64) {
            const int k = k0 + lane;
            const bool act = k < R && a.slot_last[m_lo + k] >= a.lo_round;
            const uint64_t b = __ballot(act);
            if (act) s_slot[n + __popcll(b & ((1ull << lane) - 1))] = (uint16_t)k;
            n += __popcll(b);
        }
        if (lane == 0) s_n = n;
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        // the window's slots of every topic (k_ihave_pairs decision, as k_gossip_count)
        int tot = 0;
        for (int m0 = 0; m0 < a.ring; m0 += 64)
            tot += __popcll(__ballot(m0 + lane < a.ring && a.slot_last[m0 + lane] >= a.lo_round));
        if (lane == 0 && tot > a.max_ihave) atomicOr(&a.nresp[3], 4u);
    }
    const int ns = s_n;
    const int64_t M = a.mcount[t];
    const int64_t tick_round = a.tick * a.R;
    for (int64_t j0 = (int64_t)(blockIdx.x - mctab[t]) * 1024 + wid * 64; j0 < M && ns; j0 += 256) {
        if (j0 >= (int64_t)(blockIdx.x - mctab[t] + 1) * 1024) break;
        const int64_t j = j0 + lane;
        const bool vp = j < M;
        const uint32_t p = vp ? member_peer(a, t, j) : 0u;
        const bool subp = vp && ((a.sub[p] >> t) & 1ull) && p >= a.rlo && p < a.rhi;
        uint64_t hw0 = 0, hw1 = 0, uw0 = 0, uw1 = 0;       // the member's held / unseen window slots
        for (int q0 = 0; q0 < ns; q0 += kCountBatch) {
          uint64_t cb[kCountBatch];                         // the batch's cells in flight together
#pragma unroll
          for (int b = 0; b < kCountBatch; ++b)
              cb[b] = (vp && q0 + b < ns) ? a.cs.cell[(int64_t)a.cs.cbase[m_lo + s_slot[q0 + b]] + j] : kUnseen64;
#pragma unroll
          for (int b = 0; b < kCountBatch; ++b) {
            const int q = q0 + b;
            if (q >= ns) break;                                // block-uniform
            const int k = s_slot[q];
            const uint32_t m = (uint32_t)(m_lo + k);
            const uint64_t c = cb[b];
            const bool hold = vp && holds_in_window(c, a.g, a.lo_round, tick_round, a.minv[m] != 0, p == a.morigin[m],
                                                    LAT ? a.mlat[m] : 0u);
            const bool want = subp && c == kUnseen64;
            const uint64_t kb = 1ull << (k & 63);
            if (hold) { if (k < 64) hw0 |= kb; else hw1 |= kb; }
            if (c == kUnseen64) { if (k < 64) uw0 |= kb; else uw1 |= kb; }
            const int nh = __popcll(__ballot(hold)), nw = __popcll(__ballot(want));
            if (lane == 0 && nh) atomicAdd(&s_c[k], (uint32_t)nh);
            if (lane == 0 && nw) atomicAdd(&s_c[R + k], (uint32_t)nw);
          }
        }
        if (a.ihm && vp) {
            uint64_t* o = a.ihm + (a.mmb[t] + j) * 4;
            o[0] = hw0; o[1] = hw1; o[2] = uw0; o[3] = uw1;
        }
    }
    __syncthreads();
    for (int w = threadIdx.x; w < 2 * R; w += blockDim.x)
        if (s_c[w]) atomicAdd(&gcount[(w < R ? 0 : a.ring - R) + m_lo + w], s_c[w]);
}

// waves per SIMD the member-major IHAVE walk is fitted to: round 4 measured 5
// (96 VGPRs, 25 spilled) against 4 (112): c5 gossip 96.4 -> 92.0 ms per tick; with
// the window masks (round 6) 4 is faster again (with the hub threshold and slices
// below: 86.3 -> 66.9 ms, profiles/r06_ihave_mask_ab.txt)
#ifndef GSIM_IH_WPE
#define GSIM_IH_WPE 4
#endif
#ifndef GSIM_IH_BATCH
#define GSIM_IH_BATCH 4
#endif
constexpr int kIhBatch = GSIM_IH_BATCH;   // MM walks: slots whose cells one lane loads at once
// MM hub rows (members are in peer-id order, and a power law's largest rows
// cluster at the low ids: a topic's first waves would walk dozens of hubs each,
// serially): LP 1 walks every row of at most kIhHub connections and lists the
// waves holding longer ones (IhArgs::hubw, with their slice count: one per
// 256 connections of the wave's longest row); LP 2 walks only those rows, a
// block of one wave per (listed wave, slice) -- slice s of ns taking the
// 64-edge chunks s, s + ns, ... of each row (blocks past ns exit at once)
// (128: 38.3 + 63.6 ms at c5 -- many more listed waves -- against 256: 39.4 + 11.0
// with 16 slices each, gpurun_out/r04c5h, r04c5i); round 6, once a target's ask is
// one mask load: 1024 and 8 slices (256 / 16: 86.3 ms, 512 / 8: 67.9, 1024 / 8: 66.9)
#ifndef GSIM_IH_HUB
#define GSIM_IH_HUB 1024
#endif
#ifndef GSIM_IH_SLICES
#define GSIM_IH_SLICES 8
#endif
constexpr uint32_t kIhHub = GSIM_IH_HUB;
constexpr int kIhSlices = GSIM_IH_SLICES;
#ifdef GSIM_DIAG_IH
// diagnostic build (counts and wave clocks only, results unchanged), per LP (1, 2):
// [0] push row walks, [1] push edges, [2] their gossip targets, [3] pull row walks,
// [4] pull edges, [5] their gossiping advertisers, [6] push clocks, [7] pull clocks
// (per wave), read by gsim_diag_ih_counts
__device__ unsigned long long g_ih_diag[16];
#define IH_D(...) __VA_ARGS__
#else
#define IH_D(...)
#endif
template <int W, bool LAT, bool SP, bool MM = false, int LP = 0>
__global__ __launch_bounds__(256, MM ? GSIM_IH_WPE : 1) void k_ihave(IhArgs a_, const uint32_t* gcount)
{
    const IhArgs& a = a_;
    extern __shared__ uint16_t s_act[];   // [ring] candidate slots (bit 15: push), then response staging
    __shared__ int s_n;
    if (a.nresp[3] & 4u) return;          // a truncation may apply: k_ihave_pairs
    const int wid = threadIdx.x >> 6;
    uint64_t* stage = reinterpret_cast<uint64_t*>(s_act + ((a.ring + 3) & ~3)) + wid * kRespStage;
    // LP 2: the listed wave (its block and wave) and the slice
    const uint32_t hw = LP == 2 ? a.hubw[blockIdx.x / kIhSlices] : 0u;
    const uint32_t bx = LP == 2 ? (hw & 0x07FFFFFFu) >> 2 : blockIdx.x;
    const int wsel = LP == 2 ? (int)(hw & 3u) : wid;
    const uint32_t slice = LP == 2 ? blockIdx.x % kIhSlices : 0u;
    const uint32_t nsl = LP == 2 ? (hw >> 27) + 1u : 1u;          // the wave's slice count
    if (LP == 2 && slice >= nsl) return;
    // MM: the block's topic and its 256 members [jb, jb + 256) (member-major
    // walk of a sub-ring: only the topic's slots, cells at cbase[m] + member)
    const int32_t tb = MM ? block_topic(a.mmtab, a.T, bx) : 0;
    const int64_t jb = MM ? (int64_t)(bx - a.mmtab[tb]) * 256 : 0;
    const int m_lo = MM ? tb * a.topic_slots : 0, m_hi = MM ? m_lo + a.topic_slots : a.ring;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        int n = 0;
        for (int m0 = m_lo; m0 < m_hi; m0 += 64) {
            const int m = m0 + lane;
            const bool act = m < m_hi && a.slot_last[m] >= a.lo_round && gcount[m] != 0 && gcount[a.ring + m] != 0;
            // cost model: a holder walk probes ~Dlazy cells, a receiver walk ~deg
            // (a shard's holders include its ghosts: their ghost rows are their
            // connections to its receivers)
            const bool push = act && (uint64_t)gcount[m] * 4u < (uint64_t)gcount[a.ring + m] * 32u;
            const uint64_t b = __ballot(act);
            if (act) s_act[n + __popcll(b & ((1ull << lane) - 1))] = (uint16_t)(m | (push ? 0x8000 : 0));
            n += __popcll(b);
        }
        if (lane == 0) s_n = n;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t p0 = MM ? 0 : ((int64_t)blockIdx.x * 4 + wid) * 64;   // peers p0 .. p0 + 63
    const int64_t jw = jb + wsel * 64;                                 // MM: members jw .. jw + 63
    const int nact = (MM ? jw < a.mcount[tb] : p0 < a.CN) ? s_n : 0;
    const bool vp = MM ? jw + lane < a.mcount[tb] : p0 + lane < a.CN;
    const int64_t pl = MM ? (vp ? (int64_t)member_peer(a, tb, jw + lane) : 0) : p0 + lane;
    const int grp = lane / W, gl = lane % W;
    const uint64_t gmask = group_mask<W>(grp);
    const uint64_t subp = vp ? a.sub[pl] : 0ull;
    const uint32_t rp0 = vp ? a.row_ptr[pl] : 0u;
    const uint32_t rp1 = vp ? a.row_ptr[pl + 1] : 0u;
    const bool ign_l = vp && (a.behaviour[pl] & GSIM_BEHAVE_IGNORE_IWANT);
    const uint64_t long_lanes = W < 64 ? __ballot(rp1 - rp0 > 4u * (uint32_t)W) : 0ull;
    // LP 1: rows left to LP 2; LP 2: its only rows
    const uint64_t hub_lanes = LP ? __ballot(rp1 - rp0 > kIhHub) : 0ull;
    bool had_hub = false;
    uint32_t hub_max = LP == 1 && rp1 - rp0 > kIhHub ? rp1 - rp0 : 0u;
    if constexpr (LP == 1)
        for (int o = 32; o; o >>= 1) hub_max = max(hub_max, (uint32_t)__shfl_xor((int)hub_max, o, 64));
    const int64_t tick_round = a.tick * a.R;
    int nstage = 0;
    unsigned long long n_walk = 0, n_req = 0, n_resp = 0;
    auto flush_stage = [&]() {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        uint32_t base = 0;
        if (lane == 0 && nstage) base = atomicAdd(&a.nresp[0], (uint32_t)nstage);
        base = __shfl(base, 0, 64);
        for (int q = lane; q < nstage; q += 64) {
            if ((int64_t)base + q < a.resp_cap) a.resp[base + q] = stage[q];
            else atomicOr(&a.nresp[1], 1u);
        }
        nstage = 0;
    };
    // MM: the member-major phases below walk a row once for many slots
    for (int k0 = 0; !MM && k0 < nact; k0 += kSlotBatch) {
        uint64_t cv[kSlotBatch];
#pragma unroll
        for (int b = 0; b < kSlotBatch; ++b) {
            const int k = k0 + b;
            const int64_t ci = (k < nact && vp)
                                   ? (MM ? (int64_t)a.cs.cbase[s_act[k] & 0x7FFF] + jw + lane
                                         : word_cell<SP>(a.cs, a.mtopic, s_act[k] & 0x7FFF, p0 >> 6, lane))
                                   : -1;
            cv[b] = ci >= 0 ? a.cs.cell[ci] : kUnseen64;   // no cell: not a member, nothing held or wanted
        }
#pragma unroll
        for (int b = 0; b < kSlotBatch; ++b) {
            const IhArgs& a = kernarg0(a_);   // (re-read per slot: SGPR pressure)
            const int k = k0 + b;
            if (k >= nact) break;                            // wave-uniform
            const uint32_t m = s_act[k] & 0x7FFF;
            const bool push = (s_act[k] & 0x8000) != 0;
            const int32_t t = (int32_t)a.mtopic[m];
            const uint32_t origin = a.morigin[m];
            const bool inv = a.minv[m] != 0;
            // push: lanes are holders of m (its advertisers); pull: lanes are
            // receivers that joined t and have not seen m (handleIHave's seenMessage)
            const bool me = vp && (push ? holds_in_window(cv[b], a.g, a.lo_round, tick_round, inv, (uint32_t)pl == origin,
                                                          LAT ? a.mlat[m] : 0u)
                                        : (cv[b] == kUnseen64 && ((subp >> t) & 1ull) && pl >= a.rlo && pl < a.rhi));
            const uint64_t mask = __ballot(me);
            if (!mask) continue;
            const int64_t cb_m = (int64_t)a.cs.cbase[m];
            // one chunk of a row walk: lane gl of a group of `gw` lanes takes
            // edge beg + off + gl of peer me_id's row (me_pl: its plane of t)
            auto chunk = [&](uint32_t off, uint32_t gl_, uint32_t beg, uint32_t deg, uint32_t me_id, uint32_t me_g,
                             bool ign_s, int64_t me_pl) {
                const bool v = off + gl_ < deg;
                const uint32_t e = beg + off + gl_;
                bool req = false, resp = false;
                uint32_t r = 0;
                if (push) {
                    // holder me_id walks its row: the peers it gossiped t to
                    if (v && me_pl >= 0 && a.gsel[me_pl + e]) {
                        const uint32_t p = a.col[e], re = a.rev[e];
                        // p's gate on i, p has not seen m (a shard: p one of its receivers)
                        const int64_t pci = a.cs.at(cb_m, t, p);
                        req = p >= a.rlo && p < a.rhi && a.gstate[re] && pci >= 0 && a.cs.cell[pci] == kUnseen64;
                        if (req) {
                            if (a.tr.ev) trace_iwant(a, p, me_id, m);
                            const uint64_t key = pair_key(a.seed, (uint32_t)a.tick, a.gid ? a.gid[p] : p, 0, P_PROMISE,
                                                          m, me_g);
                            atomicMin(reinterpret_cast<unsigned long long*>(&a.pcand[re]), (unsigned long long)key);
                            r = e;
                            resp = a.respond && a.gstate[e] && !ign_s && peertx_allows(a, m, e, me_id);
                        }
                    }
                } else {
                    // receiver me_id walks its row: the peers that gossiped t to it and hold m
                    if (v) {
                        const uint32_t re = a.rev[e];
                        const uint32_t i = a.col[e];
                        const uint64_t mi = smask_of(a.smask, i);        // i's emitGossip choices: its row
                        if (slot_has(mi, t) && a.gsel[slot_idx(mi, t, a.E, re)] && a.gstate[e]) {
                            const int64_t ici = a.cs.at(cb_m, t, i);
                            req = holds_in_window(ici >= 0 ? a.cs.cell[ici] : kUnseen64, a.g, a.lo_round, tick_round, inv,
                                                  i == origin, LAT ? a.mlat[m] : 0u);
                            if (req) {
                                if (a.tr.ev) trace_iwant(a, me_id, i, m);
                                const uint64_t key = pair_key(a.seed, (uint32_t)a.tick, me_g, 0, P_PROMISE, m,
                                                              a.gid ? a.gid[i] : i);
                                atomicMin(reinterpret_cast<unsigned long long*>(&a.pcand[e]), (unsigned long long)key);
                                r = re;
                                resp = a.respond && a.gstate[re] && !(a.behaviour[i] & GSIM_BEHAVE_IGNORE_IWANT) &&
                                       peertx_allows(a, m, re, i);
                            }
                        }
                    }
                }
                n_req += req;
                n_resp += resp;
                const uint64_t sb = __ballot(resp);
                if (sb) {
                    if (nstage + __popcll(sb) > kRespStage) flush_stage();
                    if (resp) stage[nstage + __popcll(sb & ((1ull << lane) - 1))] = (uint64_t)r | ((uint64_t)m << 32);
                    nstage += __popcll(sb);
                }
            };
            // rows longer than 4 groups' width are walked by the whole wave
            // afterwards, so one hub does not hold its wave's other groups
            // through its chunks
            const uint64_t longm = mask & long_lanes;
            uint64_t gm = mask & ~longm & gmask;
            while (__ballot(gm != 0)) {
                int bs = -1;
                if (gm) { bs = __ffsll((long long)gm) - 1; gm &= gm - 1; }
                const int sl = bs < 0 ? lane : bs;
                const uint32_t beg = __shfl(rp0, sl, 64), end = __shfl(rp1, sl, 64);
                const bool ign_s = __shfl(ign_l, sl, 64);
                const uint32_t me_id = MM ? (uint32_t)__shfl((int)pl, sl, 64) : (uint32_t)(p0 + (bs < 0 ? 0 : bs));
                const uint32_t me_g = a.gid ? a.gid[me_id] : me_id;   // Philox keys use global ids
                const uint64_t me_m = smask_of(a.smask, me_id);
                const int64_t me_pl = slot_has(me_m, t) ? slot_idx(me_m, t, a.E, 0) : -1;
                n_walk += (gl == 0 && bs >= 0);
                // rows longer than the group are walked in W-edge chunks (wave-uniform trip count)
                const uint32_t deg = bs >= 0 ? end - beg : 0u;
                for (uint32_t off = 0; __ballot(off < deg) != 0; off += W)
                    chunk(off, (uint32_t)gl, beg, deg, me_id, me_g, ign_s, me_pl);
            }
            for (uint64_t lm = longm; lm; lm &= lm - 1) {
                const int bs = __builtin_ctzll(lm);
                const uint32_t beg = __shfl(rp0, bs, 64), end = __shfl(rp1, bs, 64);
                const bool ign_s = __shfl(ign_l, bs, 64);
                const uint32_t me_id = MM ? (uint32_t)__shfl((int)pl, bs, 64) : (uint32_t)(p0 + bs);
                const uint32_t me_g = a.gid ? a.gid[me_id] : me_id;
                const uint64_t me_m = smask_of(a.smask, me_id);
                const int64_t me_pl = slot_has(me_m, t) ? slot_idx(me_m, t, a.E, 0) : -1;
                n_walk += (lane == 0);
                for (uint32_t off = 0; off < end - beg; off += 64)
                    chunk(off, (uint32_t)lane, beg, end - beg, me_id, me_g, ign_s, me_pl);
            }
        }
    }
    IH_D(unsigned long long d_pw = 0, d_pe = 0, d_ph = 0, d_qw = 0, d_qe = 0, d_qh = 0, d_pc = 0, d_qc = 0;)
    if constexpr (MM) {
        IH_D(const unsigned long long c_p0 = clock64();)
        // the member's held / unseen window slots (k_gossip_count_mm), else its cells below
        const bool msk = a.ihm != nullptr;
        uint64_t ih0 = 0, ih1 = 0, iu0 = 0, iu1 = 0;
        if (msk && vp) {
            const uint64_t* o = a.ihm + (a.mmb[tb] + jw + lane) * 4;
            ih0 = o[0]; ih1 = o[1]; iu0 = o[2]; iu1 = o[3];
        }
        // push slots of the block's topic, up to 64 at a time: a holder walks its
        // row once for all the slots it holds, and each peer it gossiped tb to
        // (and that is one of this shard's receivers, whose gate passes) is
        // asked about each of them (the same triples as a walk per slot).
        // With the window masks (msk) one pass takes every push slot, by
        // sub-ring index: a target's asks are (held & push) & its unseen slots,
        // one AND, and only the asked slots are visited.
        // each lane's member's plane of tb (its gossip choices), shuffled to the walking group
        int64_t own_pl = -1;
        if (vp) {
            const uint64_t om = smask_of(a.smask, (uint32_t)pl);
            own_pl = slot_has(om, tb) ? slot_idx(om, tb, a.E, 0) : -1;
        }
        uint64_t pk0 = 0, pk1 = 0;                          // msk: the push slots by sub-ring index
        if (msk) {
            for (int q = lane; q < nact; q += 64) {
                const uint16_t sa = s_act[q];
                if (!(sa & 0x8000)) continue;
                const int k = (int)(sa & 0x7FFF) - m_lo;
                if (k < 64) pk0 |= 1ull << k; else pk1 |= 1ull << (k - 64);
            }
            for (int o = 32; o; o >>= 1) {
                pk0 |= (uint64_t)__shfl_xor((long long)pk0, o, 64);
                pk1 |= (uint64_t)__shfl_xor((long long)pk1, o, 64);
            }
        }
        for (int k0 = 0; k0 < nact; k0 += msk ? nact : 64) {
            const int kn = nact - k0 < 64 ? nact - k0 : 64;
            uint64_t hm = 0, hm1 = 0;                        // msk: words 0 / 1 by sub-ring index
            if (msk) {
                if (vp) { hm = ih0 & pk0; hm1 = ih1 & pk1; }
            } else {
                for (int q = 0; q < kn; ++q) {
                    const uint16_t sa = s_act[k0 + q];
                    if (!(sa & 0x8000)) continue;                // pulled below (wave-uniform)
                    const uint32_t m = sa & 0x7FFF;
                    const uint64_t c = vp ? a.cs.cell[(int64_t)a.cs.cbase[m] + jw + lane] : kUnseen64;
                    if (vp && holds_in_window(c, a.g, a.lo_round, tick_round, a.minv[m] != 0, (uint32_t)pl == a.morigin[m],
                                              LAT ? a.mlat[m] : 0u))
                        hm |= 1ull << q;
                }
            }
            const uint64_t mask = __ballot((hm | hm1) != 0);
            if (!mask) continue;
            const int32_t t = tb;
            // one IWANT id: p (global pg) asks holder me_id over edge e for slot m
            auto ask_one = [&](bool req, uint32_t m, uint32_t p, uint32_t pg, uint32_t re, uint32_t e, uint32_t me_id,
                               uint32_t me_g, bool ign_s) {
                bool resp = false;
                if (req) {
                    if (a.tr.ev) trace_iwant(a, p, me_id, m);
                    const uint64_t key = pair_key(a.seed, (uint32_t)a.tick, pg, 0, P_PROMISE, m, me_g);
                    atomicMin(reinterpret_cast<unsigned long long*>(&a.pcand[re]), (unsigned long long)key);
                    resp = a.respond && a.gstate[e] && !ign_s && peertx_allows(a, m, e, me_id);
                }
                n_req += req;
                n_resp += resp;
                const uint64_t sb = __ballot(resp);
                if (sb) {
                    if (nstage + __popcll(sb) > kRespStage) flush_stage();
                    if (resp) stage[nstage + __popcll(sb & ((1ull << lane) - 1))] = (uint64_t)e | ((uint64_t)m << 32);
                    nstage += __popcll(sb);
                }
            };
            auto hchunk = [&](uint32_t off, uint32_t gl_, uint32_t beg, uint32_t deg, uint32_t me_id, uint32_t me_g,
                              bool ign_s, int64_t me_pl, uint64_t hmw, uint64_t hmw1) {
                const bool v = off + gl_ < deg;
                const uint32_t e = beg + off + gl_;
                uint32_t p = 0, re = 0;
                bool gs = false;
                if (v && me_pl >= 0 && a.gsel[me_pl + e]) {        // holder me_id gossiped tb to p
                    p = a.col[e];
                    re = a.rev[e];
                    gs = p >= a.rlo && p < a.rhi && a.gstate[re];  // p's gate on me_id
                    IH_D(d_ph++;)
                }
                IH_D(d_pe += v;)
                const uint32_t pg = gs ? (a.gid ? a.gid[p] : p) : 0u;
                const int64_t poff = gs ? a.cs.at(0, t, p) : -1;    // p's cell in every slot of tb
                if (msk) {
                    // the slots p is asked for: held by me_id, pushed, unseen by p
                    uint64_t r0 = 0, r1 = 0;
                    if (poff >= 0) {
                        const uint64_t* o = a.ihm + (a.mmb[t] + poff) * 4 + 2;
                        r0 = hmw & o[0];
                        r1 = hmw1 & o[1];
                    }
                    while (__ballot((r0 | r1) != 0)) {
                        int k = -1;
                        if (r0) { k = __builtin_ctzll(r0); r0 &= r0 - 1; }
                        else if (r1) { k = 64 + __builtin_ctzll(r1); r1 &= r1 - 1; }
                        ask_one(k >= 0, (uint32_t)(m_lo + (k < 0 ? 0 : k)), p, pg, re, e, me_id, me_g, ign_s);
                    }
                    return;
                }
                const uint64_t mine = gs ? hmw : 0ull;
                uint64_t uw = mine;
                for (int o = 32; o; o >>= 1) uw |= (uint64_t)__shfl_xor((long long)uw, o, 64);
                while (uw) {
                  // kIhBatch slots' cells in flight at once (nothing here writes a cell)
                  int qb[kIhBatch];
                  bool ask[kIhBatch];
                  uint64_t cvb[kIhBatch];
#pragma unroll
                  for (int b = 0; b < kIhBatch; ++b) {
                      qb[b] = uw ? __builtin_ctzll(uw) : -1;
                      if (uw) uw &= uw - 1;
                      ask[b] = qb[b] >= 0 && ((mine >> qb[b]) & 1ull) && poff >= 0;
                      cvb[b] = ask[b] ? a.cs.cell[(int64_t)a.cs.cbase[s_act[k0 + qb[b]] & 0x7FFF] + poff] : 0ull;
                  }
#pragma unroll
                  for (int b = 0; b < kIhBatch; ++b) {
                    const int q = qb[b];
                    if (q < 0) break;                                // wave-uniform
                    ask_one(ask[b] && cvb[b] == kUnseen64, s_act[k0 + q] & 0x7FFF, p, pg, re, e, me_id, me_g, ign_s);
                  }
                }
            };
            had_hub = had_hub || (mask & hub_lanes) != 0;
            const uint64_t longm = LP == 2 ? (mask & hub_lanes) : LP == 1 ? (mask & long_lanes & ~hub_lanes)
                                                                           : (mask & long_lanes);
            uint64_t gm = LP == 2 ? 0ull : (mask & ~long_lanes & gmask);
            while (__ballot(gm != 0)) {
                int bs = -1;
                if (gm) { bs = __ffsll((long long)gm) - 1; gm &= gm - 1; }
                const int sl = bs < 0 ? lane : bs;
                const uint32_t beg = __shfl(rp0, sl, 64), end = __shfl(rp1, sl, 64);
                const bool ign_s = __shfl(ign_l, sl, 64);
                const uint32_t me_id = (uint32_t)__shfl((int)pl, sl, 64);
                const uint64_t hmw = bs < 0 ? 0ull : (uint64_t)__shfl((long long)hm, sl, 64);
                const uint64_t hmw1 = bs < 0 ? 0ull : (uint64_t)__shfl((long long)hm1, sl, 64);
                const uint32_t me_g = a.gid ? a.gid[me_id] : me_id;
                const int64_t me_pl = (int64_t)__shfl((long long)own_pl, sl, 64);
                n_walk += (gl == 0 && bs >= 0);
                IH_D(d_pw += (gl == 0 && bs >= 0);)
                const uint32_t deg = bs >= 0 ? end - beg : 0u;
                for (uint32_t off = 0; __ballot(off < deg) != 0; off += W)
                    hchunk(off, (uint32_t)gl, beg, deg, me_id, me_g, ign_s, me_pl, hmw, hmw1);
            }
            for (uint64_t lm = longm; lm; lm &= lm - 1) {
                const int bs = __builtin_ctzll(lm);
                const uint32_t beg = __shfl(rp0, bs, 64), end = __shfl(rp1, bs, 64);
                const bool ign_s = __shfl(ign_l, bs, 64);
                const uint32_t me_id = (uint32_t)__shfl((int)pl, bs, 64);
                const uint64_t hmw = (uint64_t)__shfl((long long)hm, bs, 64);
                const uint64_t hmw1 = (uint64_t)__shfl((long long)hm1, bs, 64);
                const uint32_t me_g = a.gid ? a.gid[me_id] : me_id;
                const int64_t me_pl = (int64_t)__shfl((long long)own_pl, bs, 64);
                n_walk += (lane == 0 && slice == 0);
                IH_D(d_pw += (lane == 0 && slice == 0);)
                for (uint32_t off = slice * 64; off < end - beg; off += 64 * nsl)
                    hchunk(off, (uint32_t)lane, beg, end - beg, me_id, me_g, ign_s, me_pl, hmw, hmw1);
            }
        }
        // pull slots of the block's topic, up to 64 at a time: a receiver walks
        // its row once for all the slots it wants (not once per slot), and an
        // edge whose advertiser gossiped tb to it asks for each wanted slot
        // the advertiser holds (the same (receiver, advertiser, message)
        // triples as a walk per slot)
        IH_D(const unsigned long long c_p1 = clock64(); d_pc += c_p1 - c_p0;)
        const bool rcv = vp && ((subp >> tb) & 1ull) && pl >= a.rlo && pl < a.rhi;
        for (int k0 = 0; k0 < nact; k0 += 64) {
            const int kn = nact - k0 < 64 ? nact - k0 : 64;
            uint64_t wm = 0;
            for (int q = 0; q < kn; ++q) {
                const uint16_t sa = s_act[k0 + q];
                if (sa & 0x8000) continue;                   // pushed above (wave-uniform)
                if (msk) {
                    if (rcv && bit128(iu0, iu1, (int)(sa & 0x7FFF) - m_lo)) wm |= 1ull << q;
                    continue;
                }
                const uint64_t c = rcv ? a.cs.cell[(int64_t)a.cs.cbase[sa & 0x7FFF] + jw + lane] : 0ull;
                if (rcv && c == kUnseen64) wm |= 1ull << q;
            }
            const uint64_t mask = __ballot(wm != 0);
            if (!mask) continue;
            const int32_t t = tb;
            auto pchunk = [&](uint32_t off, uint32_t gl_, uint32_t beg, uint32_t deg, uint32_t me_id, uint32_t me_g, uint64_t wmw) {
                const bool v = off + gl_ < deg;
                const uint32_t e = beg + off + gl_;
                uint32_t re = 0, i = 0;
                bool gs = false;
                if (v) {
                    re = a.rev[e];
                    i = a.col[e];
                    const uint64_t mi = smask_of(a.smask, i);        // i's emitGossip choices: its row
                    gs = slot_has(mi, t) && a.gsel[slot_idx(mi, t, a.E, re)] && a.gstate[e];
                }
                IH_D(d_qe += v; d_qh += gs;)
                const uint64_t mine = gs ? wmw : 0ull;
                uint64_t uw = mine;                                  // the slots some lane asks about
                for (int o = 32; o; o >>= 1) uw |= (uint64_t)__shfl_xor((long long)uw, o, 64);
                const uint32_t ig = gs ? (a.gid ? a.gid[i] : i) : 0u;
                const int64_t ioff = gs ? a.cs.at(0, t, i) : -1;    // i's cell in every slot of tb
                uint64_t ah0 = 0, ah1 = 0;                          // ... or its held window slots
                if (msk && ioff >= 0) {
                    const uint64_t* o = a.ihm + (a.mmb[t] + ioff) * 4;
                    ah0 = o[0]; ah1 = o[1];
                }
                while (uw) {
                  // kIhBatch slots' cells in flight at once (nothing here writes a cell)
                  int qb[kIhBatch];
                  uint64_t cvb[kIhBatch];
#pragma unroll
                  for (int b = 0; b < kIhBatch; ++b) {
                      qb[b] = uw ? __builtin_ctzll(uw) : -1;
                      if (uw) uw &= uw - 1;
                      const bool ask = qb[b] >= 0 && ((mine >> qb[b]) & 1ull) && ioff >= 0;
                      const uint32_t mb = ask ? s_act[k0 + qb[b]] & 0x7FFF : 0u;
                      // a held slot: its cell (msk: the mask stands in, read as held below)
                      cvb[b] = !ask ? kUnseen64 : msk ? (bit128(ah0, ah1, (int)mb - m_lo) ? 1ull : kUnseen64)
                                                      : a.cs.cell[(int64_t)a.cs.cbase[mb] + ioff];
                  }
#pragma unroll
                  for (int b = 0; b < kIhBatch; ++b) {
                    const int q = qb[b];
                    if (q < 0) break;                                // wave-uniform
                    const uint32_t m = s_act[k0 + q] & 0x7FFF;
                    bool req = false, resp = false;
                    if ((mine >> q) & 1ull) {
                        req = msk ? cvb[b] != kUnseen64
                                  : holds_in_window(cvb[b], a.g, a.lo_round, tick_round,
                                                    a.minv[m] != 0, i == a.morigin[m], LAT ? a.mlat[m] : 0u);
                        if (req) {
                            if (a.tr.ev) trace_iwant(a, me_id, i, m);
                            const uint64_t key = pair_key(a.seed, (uint32_t)a.tick, me_g, 0, P_PROMISE, m, ig);
                            atomicMin(reinterpret_cast<unsigned long long*>(&a.pcand[e]), (unsigned long long)key);
                            resp = a.respond && a.gstate[re] && !(a.behaviour[i] & GSIM_BEHAVE_IGNORE_IWANT) &&
                                   peertx_allows(a, m, re, i);
                        }
                    }
                    n_req += req;
                    n_resp += resp;
                    const uint64_t sb = __ballot(resp);
                    if (sb) {
                        if (nstage + __popcll(sb) > kRespStage) flush_stage();
                        if (resp) stage[nstage + __popcll(sb & ((1ull << lane) - 1))] = (uint64_t)re | ((uint64_t)m << 32);
                        nstage += __popcll(sb);
                    }
                  }
                }
            };
            had_hub = had_hub || (mask & hub_lanes) != 0;
            const uint64_t longm = LP == 2 ? (mask & hub_lanes) : LP == 1 ? (mask & long_lanes & ~hub_lanes)
                                                                           : (mask & long_lanes);
            uint64_t gm = LP == 2 ? 0ull : (mask & ~long_lanes & gmask);
            while (__ballot(gm != 0)) {
                int bs = -1;
                if (gm) { bs = __ffsll((long long)gm) - 1; gm &= gm - 1; }
                const int sl = bs < 0 ? lane : bs;
                const uint32_t beg = __shfl(rp0, sl, 64), end = __shfl(rp1, sl, 64);
                const uint32_t me_id = (uint32_t)__shfl((int)pl, sl, 64);
                const uint64_t wmw = bs < 0 ? 0ull : (uint64_t)__shfl((long long)wm, sl, 64);
                const uint32_t me_g = a.gid ? a.gid[me_id] : me_id;
                n_walk += (gl == 0 && bs >= 0);
                IH_D(d_qw += (gl == 0 && bs >= 0);)
                const uint32_t deg = bs >= 0 ? end - beg : 0u;
                for (uint32_t off = 0; __ballot(off < deg) != 0; off += W) pchunk(off, (uint32_t)gl, beg, deg, me_id, me_g, wmw);
            }
            for (uint64_t lm = longm; lm; lm &= lm - 1) {
                const int bs = __builtin_ctzll(lm);
                const uint32_t beg = __shfl(rp0, bs, 64), end = __shfl(rp1, bs, 64);
                const uint32_t me_id = (uint32_t)__shfl((int)pl, bs, 64);
                const uint64_t wmw = (uint64_t)__shfl((long long)wm, bs, 64);
                const uint32_t me_g = a.gid ? a.gid[me_id] : me_id;
                n_walk += (lane == 0 && slice == 0);
                IH_D(d_qw += (lane == 0 && slice == 0);)
                for (uint32_t off = slice * 64; off < end - beg; off += 64 * nsl)
                    pchunk(off, (uint32_t)lane, beg, end - beg, me_id, me_g, wmw);
            }
        }
        IH_D(d_qc += clock64() - c_p1;)
        if constexpr (LP == 1) {
            if (had_hub && lane == 0) {
                // every slice (one per 256 connections of the longest row made fewer,
                // longer blocks: 25.3 against 11.0 ms, gpurun_out/r04c5j)
                const uint32_t ns = (uint32_t)kIhSlices;
                (void)hub_max;
                a.hubw[atomicAdd(a.hubn, 1u)] = (blockIdx.x * 4u + (uint32_t)wid) | ((ns - 1u) << 27);
            }
        }
    }
    flush_stage();
#ifdef GSIM_DIAG_IH
    if (MM && LP) {
        unsigned long long* dg = g_ih_diag + (LP == 2 ? 8 : 0);
        const unsigned long long v6[6] = {wave_sum_u64(d_pw), wave_sum_u64(d_pe), wave_sum_u64(d_ph),
                                          wave_sum_u64(d_qw), wave_sum_u64(d_qe), wave_sum_u64(d_qh)};
        if (lane == 0) {
            for (int q = 0; q < 6; ++q) if (v6[q]) atomicAdd(&dg[q], v6[q]);
            atomicAdd(&dg[6], d_pc);
            atomicAdd(&dg[7], d_qc);
        }
    }
#endif
    n_walk = wave_sum_u64(n_walk);
    n_req = wave_sum_u64(n_req);
    n_resp = wave_sum_u64(n_resp);
    if (lane == 0 && (n_walk | n_req)) {
        atomicAdd(&a.gstats[0], n_walk);
        atomicAdd(&a.gstats[1], n_req);
        atomicAdd(&a.gstats[2], n_resp);
    }
}

// handleIHave when a MaxIHaveLength truncation may apply (the window holds
// more than MaxIHaveLength slots: nresp[3] bit 2).  One wave per receiver,
// walking its (receiver, advertiser) pairs in row order, as the oracle does
// (oracle_gossip.c orc_gossip_ihave):
//   * an advertiser whose window for topic t holds more than MaxIHaveLength
//     ids sends this receiver a random MaxIHaveLength-subset of it
//     (emitGossip's per-peer shuffle, gossipsub.go:1763-1772);
//   * an IWANT of more than MaxIHaveLength ids asks for a random
//     MaxIHaveLength of them (handleIHave, gossipsub.go:679-690), and the
//     promise is one of those (AddPromise, gossip_tracer.go:48-64).
// A random subset is the MaxIHaveLength smallest Philox keys; keys are unique
// (their low word is the slot), so it is {key <= tau} for the
// MaxIHaveLength-th smallest key tau, found by a binary search over the key
// value (64 counting passes over the window: a path for rare, huge windows).
constexpr int kPairTopics = 64;

template <bool LAT>
__global__ __launch_bounds__(256) void k_ihave_pairs(IhArgs a)
{
    extern __shared__ uint16_t s_act[];   // [ring] window slots, then per wave: staging, tau[64], count[64]
    __shared__ int s_n;
    if (!(a.nresp[3] & 4u)) return;       // k_ihave handles this stage
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint64_t* base = reinterpret_cast<uint64_t*>(s_act + ((a.ring + 3) & ~3));
    uint64_t* stage = base + wid * kRespStage;
    uint64_t* s_tau = base + 4 * kRespStage + wid * kPairTopics;
    uint32_t* s_cnt = reinterpret_cast<uint32_t*>(base + 4 * kRespStage + 4 * kPairTopics) + wid * kPairTopics;
    if (threadIdx.x < 64) {
        int n = 0;
        for (int m0 = 0; m0 < a.ring; m0 += 64) {
            const int m = m0 + lane;
            const bool act = m < a.ring && a.slot_last[m] >= a.lo_round;
            const uint64_t b = __ballot(act);
            if (act) s_act[n + __popcll(b & ((1ull << lane) - 1))] = (uint16_t)m;
            n += __popcll(b);
        }
        if (lane == 0) s_n = n;
    }
    __syncthreads();
    const int ns = s_n;
    const uint32_t L = (uint32_t)a.max_ihave;
    const int64_t tick_round = a.tick * a.R;
    int nstage = 0;
    unsigned long long n_walk = 0, n_req = 0, n_resp = 0;
    auto flush_stage = [&]() {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        uint32_t b0 = 0;
        if (lane == 0 && nstage) b0 = atomicAdd(&a.nresp[0], (uint32_t)nstage);
        b0 = __shfl(b0, 0, 64);
        for (int q = lane; q < nstage; q += 64) {
            if ((int64_t)b0 + q < a.resp_cap) a.resp[b0 + q] = stage[q];
            else atomicOr(&a.nresp[1], 1u);
        }
        nstage = 0;
    };
    auto lds_sync = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // the L-th smallest key over the window slots k with sel(k, &key)
    auto kth_key = [&](auto sel) -> uint64_t {
        uint64_t lo = 0, hi = ~0ull;
        while (lo < hi) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            uint32_t c = 0;
            for (int k0 = 0; k0 < ns; k0 += 64) {
                const int k = k0 + lane;
                uint64_t key = 0;
                c += (uint32_t)__popcll(__ballot(k < ns && sel(k, key) && key <= mid));
            }
            if (c >= L) hi = mid; else lo = mid + 1;
        }
        return lo;
    };
    for (int64_t pc = (int64_t)blockIdx.x * 4 + wid; pc < a.CN; pc += (int64_t)gridDim.x * 4) {
        const uint32_t p = (uint32_t)pc;
        if (p < a.rlo || p >= a.rhi) continue;                    // receivers: owned peers
        const uint64_t subp = a.sub[p];
        const uint32_t beg = a.row_ptr[p], end = a.row_ptr[p + 1];
        const uint32_t p_g = a.gid ? a.gid[p] : p;
        for (uint32_t e = beg; e < end; ++e) {
            if (!a.gstate[e]) continue;                           // IHAVE from a peer below gossipThreshold
            const uint32_t re = a.rev[e], i = a.col[e];
            // topics i gossiped to p that p joined (gs.mesh[topic] exists); i's choices sit in its row
            const uint64_t mi = smask_of(a.smask, i);
            const bool tb = lane < a.T && ((subp >> lane) & 1ull) && slot_has(mi, lane) &&
                            a.gsel[slot_idx(mi, lane, a.E, re)];
            const uint64_t tmask = __ballot(tb);
            if (!tmask) continue;
            n_walk += (lane == 0);
            const uint32_t i_g = a.gid ? a.gid[i] : i;
            const uint32_t origin_ign = a.behaviour[i] & GSIM_BEHAVE_IGNORE_IWANT;
            auto holds = [&](uint32_t m) {
                return holds_in_window(a.cs.get(m, (int32_t)a.mtopic[m], i), a.g, a.lo_round, tick_round, a.minv[m] != 0,
                                       i == a.morigin[m], LAT ? a.mlat[m] : 0u);
            };
            // GetGossipIDs(topic) of i: ids per topic
            s_cnt[lane] = 0;
            lds_sync();
            for (int k0 = 0; k0 < ns; k0 += 64) {
                const int k = k0 + lane;
                if (k < ns) {
                    const uint32_t m = s_act[k];
                    const int t = (int)a.mtopic[m];
                    if (((tmask >> t) & 1ull) && holds(m)) atomicAdd(&s_cnt[t], 1u);
                }
            }
            lds_sync();
            const uint64_t omask = __ballot(s_cnt[lane] > L) & tmask;
            for (uint64_t om = omask; om; om &= om - 1) {
                const int t = __ffsll((long long)om) - 1;
                const uint64_t tau = kth_key([&](int k, uint64_t& key) {
                    const uint32_t m = s_act[k];
                    if ((int)a.mtopic[m] != t || !holds(m)) return false;
                    key = pair_key(a.seed, (uint32_t)a.tick, i_g, (uint32_t)t, P_IHAVE_TRUNC, m, p_g);
                    return true;
                });
                if (lane == 0) s_tau[t] = tau;
            }
            lds_sync();
            // the ids i advertised to p and p has not seen
            auto wanted = [&](uint32_t m) {
                const int t = (int)a.mtopic[m];
                if (!((tmask >> t) & 1ull) || a.cs.get(m, t, p) != kUnseen64 || !holds(m)) return false;
                return s_cnt[t] <= L ||
                       pair_key(a.seed, (uint32_t)a.tick, i_g, (uint32_t)t, P_IHAVE_TRUNC, m, p_g) <= s_tau[t];
            };
            uint32_t nw = 0;
            for (int k0 = 0; k0 < ns; k0 += 64) {
                const int k = k0 + lane;
                nw += (uint32_t)__popcll(__ballot(k < ns && wanted(s_act[k])));
            }
            if (nw == 0) continue;
            uint64_t tau_w = ~0ull;
            if (nw > L)
                tau_w = kth_key([&](int k, uint64_t& key) {
                    const uint32_t m = s_act[k];
                    if (!wanted(m)) return false;
                    key = pair_key(a.seed, (uint32_t)a.tick, p_g, 0, P_IWANT, m, i_g);
                    return true;
                });
            uint64_t pmin = ~0ull;
            for (int k0 = 0; k0 < ns; k0 += 64) {
                const int k = k0 + lane;
                const uint32_t m = k < ns ? s_act[k] : 0u;
                const bool ask = k < ns && wanted(m) &&
                                 (nw <= L || pair_key(a.seed, (uint32_t)a.tick, p_g, 0, P_IWANT, m, i_g) <= tau_w);
                bool resp = false;
                if (ask) {
                    if (a.tr.ev) trace_iwant(a, p, i, m);
                    const uint64_t key = pair_key(a.seed, (uint32_t)a.tick, p_g, 0, P_PROMISE, m, i_g);
                    pmin = key < pmin ? key : pmin;
                    // handleIWant at i: its gate on p, IWANT-ignoring behaviour, GetForPeer's count
                    resp = a.respond && a.gstate[re] && !origin_ign && peertx_allows(a, m, re, i);
                }
                n_req += ask;
                n_resp += resp;
                const uint64_t sb = __ballot(resp);
                if (sb) {
                    if (nstage + __popcll(sb) > kRespStage) flush_stage();
                    if (resp) stage[nstage + __popcll(sb & ((1ull << lane) - 1))] = (uint64_t)re | ((uint64_t)m << 32);
                    nstage += __popcll(sb);
                }
            }
            for (int o = 32; o > 0; o >>= 1) {
                const uint64_t x = __shfl_xor(pmin, o, 64);
                pmin = x < pmin ? x : pmin;
            }
            if (lane == 0) atomicMin(reinterpret_cast<unsigned long long*>(&a.pcand[e]), (unsigned long long)pmin);
        }
    }
    flush_stage();
    n_walk = wave_sum_u64(n_walk);
    n_req = wave_sum_u64(n_req);
    n_resp = wave_sum_u64(n_resp);
    if (lane == 0 && (n_walk | n_req)) {
        atomicAdd(&a.gstats[0], n_walk);
        atomicAdd(&a.gstats[1], n_req);
        atomicAdd(&a.gstats[2], n_resp);
    }
}

// AddPromise (gossip_tracer.go:48-75): the one tracked id of each IWANT,
// unless the same (id, peer) promise is still pending.
__global__ __launch_bounds__(256) void k_promise_insert(uint64_t* pcand, uint32_t* prom, int32_t P, int32_t idx,
                                                        int64_t E)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) {
        const uint64_t key = pcand[e];
        if (key == ~0ull) continue;
        pcand[e] = ~0ull;
        const uint32_t slot = (uint32_t)key;
        bool exists = false;
        for (int q = 0; q < P; ++q) exists |= prom[(int64_t)q * E + e] == slot;
        if (!exists) prom[(int64_t)idx * E + e] = slot;
    }
}

// One pending meshMessageDeliveries increment of record ir: a byte add on
// the containing word; the add that makes kMcntSpill pending moves them to
// meshd.  Increments are x -> min(x + 1, cap) one after the other until the
// next refresh applies the rest, so how they are grouped into spills does not
// change the result; fewer than 256 - kMcntSpill copies of one record arrive
// in one launch, so the byte never carries into its neighbour.
constexpr uint32_t kMcntSpill = 128;
constexpr int kPubTicks = 16;      // publication window of the mcnt_fast bound (>= HistoryLength + 3)
__device__ __forceinline__ void atomic_mcnt_inc(uint8_t* mcnt, int64_t ir, double* meshd, double cap, bool fast = false)
{
    uint32_t* w = reinterpret_cast<uint32_t*>(mcnt + (ir & ~(int64_t)3));
    const int sh = (int)(ir & 3) * 8;
    if (fast) {                      // bounded pending increments: no spill to watch for
        __hip_atomic_fetch_add(w, 1u << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const uint32_t old = atomicAdd(w, 1u << sh);
    if (((old >> sh) & 0xFFu) != kMcntSpill - 1u) return;
    atomicSub(w, kMcntSpill << sh);
    unsigned long long* q = reinterpret_cast<unsigned long long*>(meshd);
    unsigned long long o = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        const double x = apply_incs(__longlong_as_double((long long)o), kMcntSpill, cap);
        const unsigned long long nx = (unsigned long long)__double_as_longlong(x);
        const unsigned long long pv = atomicCAS(q, o, nx);
        if (pv == o) break;
        o = pv;
    }
}

// One copy of slot m on record r (the receiver col[r]'s record of the sender,
// the row owner): AcceptFrom, the peer gater, the claim of the receiver's
// cell (the lowest edge wins), the record's counters -- k_send_tm's rules for
// a copy that arrives listed (k_gossip_deliver) or as a bit (k_xbits_deliver).
// A record can receive several copies in one launch: counters are atomic.
__device__ __forceinline__ void listed_copy(const RoundArgs& a, uint32_t r, uint32_t m, const uint32_t* owner,
                                            uint32_t par, uint32_t claim_hi, ctp_t tpa, unsigned long long& n_acc,
                                            unsigned long long& n_gray, unsigned long long& n_first, uint32_t* s_new2,
                                            bool iwant_rpc)
{
    const uint8_t ds = a.dstate[r];
    if (!(ds & GSIM_DS_ACCEPT)) { n_gray++; return; }        // AcceptFrom
    const uint32_t p = a.col[r];
    // the sender (row owner) is read only where it matters: topic slots,
    // the gater, the trace, a claim (most copies are plain duplicates)
    const bool need_i = a.smask || a.gt.act || a.tr.on(p);
    uint32_t i = need_i ? owner[r] : 0xFFFFFFFFu;
    // the peer gater (gater_accept): one draw per IWANT answer RPC -- (round,
    // receiver, sender), the slot left out (AcceptFrom runs per RPC, pubsub.go);
    // a shard's pushed copies are forwarded messages, one RPC each
    if (a.gt.act && !gater_accept(a, p, r, iwant_rpc ? kGaterRpcSlot : m, i)) return;
    if (a.subdyn && !((a.sub[p] >> (int32_t)a.mtopic[m]) & 1ull)) return;   // a topic p left
    if (a.gt.act) gater_copy(a, r, a.minv[m] == GSIM_VERDICT_SIGNATURE);
    n_acc++;
    const int32_t t = (int32_t)a.mtopic[m];
    const ctp_t tp = tpa + t;
    const uint8_t vd = a.minv[m];
    if (a.tr.on(p))
        a.tr.push(round_time(a, a.g), ((uint64_t)a.g << 32) | m, p, i, t,
                  vd != GSIM_VERDICT_SIGNATURE ? kTraceCopy : (uint8_t)GSIM_TRACE_REJECT_MESSAGE, vd);
    const bool inv = vd != GSIM_VERDICT_ACCEPT;
    const bool pen = verdict_penalises(vd);
    const uint64_t mi = smask_of(a.smask, i);               // the record sits in the sender's row
    const int64_t ir = slot_idx(mi, t, a.E, r);
    const bool sc = tp->scored && (ds & GSIM_DS_TRACKED) && slot_has(mi, t);
    const uint8_t tf = a.tflags[ir];
    const int64_t window = tp->mesh_message_deliveries_window_ns;
    const uint32_t L = a.mlat ? a.mlat[m] : 0u;
    // committed before this round and the cell's round cannot matter (as
    // k_send_tm's known copies): a duplicate, credited without the cell
    if (!L && ((a.seenbm[(int64_t)m * a.nw + (p >> 6)] >> (p & 63)) & 1ull)) {
        const bool wa = window >= 0 && a.now - round_time(a, a.mpub[m]) <= window;
        if (wa || !sc || inv || !(tf & GSIM_TF_IN_MESH)) {
            if (!sc) return;
            if (pen) { atomicAdd(&a.invalid[ir], 1.0); inv_mark(a); }
            else if (!inv && (tf & GSIM_TF_IN_MESH))         // wa: within the window
                atomic_mcnt_inc(a.mcnt, ir, &a.meshd[ir], tp->mesh_message_deliveries_cap, a.mcnt_fast);
            return;
        }
    }
    const int64_t pci = a.cs.idx(m, t, p);      // p wanted it: a member of t
    if (pci < 0) return;
    uint64_t* cellp = a.cs.cell + pci;
    const uint64_t c = *cellp;
    const uint32_t hi = (uint32_t)(c >> 32);
    int64_t seen_round = -1;               // completion round (k_send_tm)
    if (c != kUnseen64) {
        if (!(hi & kClaim)) seen_round = hi;
        else if (((hi >> 30) & 1u) != par) seen_round = a.g - 1 + L;
    }
    if (vd != GSIM_VERDICT_SIGNATURE && seen_round < 0 && (c == kUnseen64 || (hi & kEdgeMask) > r)) {
        if (!need_i) i = owner[r];
        uint32_t lo = i;
        if (sc && !inv) {
            lo |= kCreditFirst;
            if (window < 0 && (tf & GSIM_TF_IN_MESH)) lo |= kCreditMesh;
        }
        const uint64_t v = ((uint64_t)(claim_hi | r) << 32) | lo;
        const uint64_t prev = __hip_atomic_fetch_min(cellp, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == kUnseen64) {
            n_first++;
            atomicOr(&s_new2[m >> 5], 1u << (m & 31));
            if (a.clist) {
                const uint32_t sq = blockIdx.x % kClSub;
                const uint32_t q = atomicAdd(&a.clist_n[sq * kClStride], 1u);
                if ((int64_t)q < a.clist_cap)
                    a.clist[(int64_t)sq * a.clist_cap + q] = cl_entry(a, p, m, cellp - a.cs.cell, (int64_t)a.cs.cbase[m]);
                else atomicOr(&a.clist_n[kClSub * kClStride], 1u);
            }
        }
    }
    if (L && vd != GSIM_VERDICT_SIGNATURE && (seen_round < 0 || seen_round > a.g)) {
        // the lanes here push together (ballots over the active lanes)
        const bool q = tp->scored && (pen || !inv);
        vq_push_wave(a, q ? (int)((seen_round < 0 ? a.g + L : seen_round) & (kVqPlanes - 1)) : -1,
                     vq_entry(r, t, pen ? kVqInv : kVqDup));
        return;
    }
    if (!sc) return;
    if (pen) {
        atomicAdd(&a.invalid[ir], 1.0);                           // markInvalidMessageDelivery
        inv_mark(a);
    } else if (!inv && (tf & GSIM_TF_IN_MESH)) {
        const bool in_window = seen_round >= 0 ? (a.now - round_time(a, seen_round) <= window) : (window >= 0);
        if (in_window) atomic_mcnt_inc(a.mcnt, ir, &a.meshd[ir], tp->mesh_message_deliveries_cap, a.mcnt_fast);
    }
}

// The list-driven send (member-compacted cells): round
// g's forwarders come as a list (Deliver::d_flist: the commit of round g-1's
// claims and round g-1's publications), so a round with a sparse frontier
// costs its forwarders' edges, not a scan of every active slot's fresh bits
// in 1024-peer chunks with block-wide scans per slot layer (c5: DESIGN §4.2).
// A block takes 256 entries, lays their walks out (a block scan of the walk
// lengths) and runs one thread per edge, kLsP edges per thread in flight.
// Each copy follows k_send_tm's rules (AcceptFrom, the claim of the receiver's
// cell -- the lowest edge wins --, the score tracer); the entries of one
// sender (its slots of a topic) may sit in different blocks, so its records
// take atomic updates (atomic_mcnt_inc, the exact +1 steps in any order, as
// listed_copy's).  Configurations with validation latency, the peer gater or
// the trace keep the scan, and so do shards on the pull exchange; shards with
// the copy push walk the list too (a ghost receiver's copy sets its bit, as in
// k_send_tm<PUSH>) -- flist_allowed.
constexpr int kLsP = 2;
constexpr int kLsB = 256;
__global__ __launch_bounds__(kLsB) void k_send_list(RoundArgs a_)
{
    const RoundArgs& a = a_;
    extern __shared__ uint32_t s_new2[];                     // [ring/32] slots with a new claim
    __shared__ uint32_t s_off[kLsB + 1];                     // first flattened edge of each entry
    __shared__ uint32_t s_x[kLsB], s_m[kLsB], s_from[kLsB], s_beg[kLsB], s_pl[kLsB];
    __shared__ uint64_t s_msk[kLsB];
    __shared__ uint64_t s_cl[kLsB * kLsP];
    __shared__ uint32_t s_wsum[kLsB / 64];
    __shared__ unsigned long long s_stats[4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int par = (int)(a.g & 1);
    if (a.fst[kFstBad + par]) return;                        // incomplete: k_send_tm scans the fresh bits
    const int64_t n = min((int64_t)a.fst[par * kFstStride], a.flist_cap);
    const uint64_t* fl = a.flist + (int64_t)par * a.flist_cap;
    for (int w = tid; w < (a.ring + 31) / 32; w += kLsB) s_new2[w] = 0;
    if (tid < 4) s_stats[tid] = 0;
    __syncthreads();
    const uint32_t claim_hi = kClaim | ((uint32_t)par << 30);
    unsigned long long n_acc = 0, n_gray = 0, n_first = 0;
    for (int64_t c0 = (int64_t)blockIdx.x * kLsB; c0 < n; c0 += (int64_t)gridDim.x * kLsB) {   // block-uniform
        const RoundArgs& a = kernarg0(a_);
        uint32_t len = 0, x = 0, m = 0, from = kPeerMask, beg = 0, pl = 0;
        uint64_t msk = 0;
        if (c0 + tid < n) {
            const uint64_t v = fl[c0 + tid];
            x = fl_x(a, v);
            m = fl_m(a, v);
            const int32_t t = (int32_t)a.mtopic[m];
            const uint32_t origin = a.morigin[m];
            // the origin's fresh bit (k_publish) is taken here; on shards every
            // entry's (the commit also set them, for the holder accumulation)
            if ((v & kFlOrigin) || a.sharded)
                atomicAnd(reinterpret_cast<unsigned long long*>(a.fresh + (int64_t)m * a.nw + (x >> 6)), ~(1ull << (x & 63)));
            if (a.fl_from) {
                from = fl_from_of(v);
            } else {
                const int64_t xc = a.cs.at((int64_t)a.cs.cbase[m], t, x);
                from = xc >= 0 ? (uint32_t)a.cs.cell[xc] & kPeerMask : kPeerMask;
            }
            const uint64_t xm = smask_of(a.smask, x);
            pl = (uint32_t)__popcll(xm & ((1ull << t) - 1ull));
            const uint32_t rb = a.row_ptr[x], deg = a.row_ptr[x + 1] - rb;
            if (!slot_has(xm, t) || a.g == 0) {
                // no state for t in x's row: nothing is sent (cannot happen)
            } else if (deg <= 64 && x != origin) {
                msk = a.mmask[(int64_t)t * a.N + x];
                beg = rb;
                len = (uint32_t)__popcll(msk);
            } else if (a.hlist && x != origin && a.hlist[((int64_t)a.hidx[x] * a.T + t) * (1 + kHubMesh)] != 0xFFFFFFFFu) {
                const uint32_t lo_ = (uint32_t)(((int64_t)a.hidx[x] * a.T + t) * (1 + kHubMesh));
                beg = kHubList | (lo_ + 1u);
                len = a.hlist[lo_];
            } else {
                beg = rb;
                len = deg;
            }
        }
        // exclusive scan of the walk lengths
        uint32_t inc = len;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) s_wsum[wid] = inc;
        __syncthreads();
        uint32_t wbase = 0, total = 0;
        for (int q = 0; q < kLsB / 64; ++q) {
            if (q < wid) wbase += s_wsum[q];
            total += s_wsum[q];
        }
        s_off[tid] = wbase + inc - len;
        if (tid == 0) s_off[kLsB] = total;
        s_x[tid] = x; s_m[tid] = m; s_from[tid] = from; s_beg[tid] = beg; s_msk[tid] = msk; s_pl[tid] = pl;
        __syncthreads();
        for (uint32_t f0 = 0; f0 < total; f0 += kLsB * kLsP) {
            const RoundArgs& a = kernarg0(a_);   // (re-read per iteration: SGPR pressure)
            uint32_t jv[kLsP], ev[kLsP], iv[kLsP], qv[kLsP], xq[kLsP];
            int64_t pv[kLsP];
            uint8_t mfv[kLsP], dsv[kLsP], tfv[kLsP];
            bool vv[kLsP], mk[kLsP], rem[kLsP];
            uint64_t xbk[kLsP], xbv[kLsP];     // push: a remote copy's xbits word (~0: none) and bit
#pragma unroll
            for (int u = 0; u < kLsP; ++u) {
                const uint32_t fi = f0 + (uint32_t)(u * kLsB + tid);
                vv[u] = fi < total;
                int l = 0, r = kLsB;
                while (r - l > 1) {                              // the entry whose walk holds edge fi
                    const int mid = (l + r) >> 1;
                    if (s_off[mid] <= fi) l = mid; else r = mid;
                }
                qv[u] = (uint32_t)l;
                const uint32_t k = fi - s_off[l];
                const uint64_t mq = s_msk[l];
                const uint32_t bq = s_beg[l];
                jv[u] = s_x[l];
                mk[u] = mq != 0 || (bq & kHubList);
                const int32_t t = (int32_t)a.mtopic[s_m[l]];
                pv[u] = (a.smask ? (int64_t)s_pl[l] : (int64_t)t) * a.E;
                if (!vv[u]) ev[u] = 0;
                else if (mq) ev[u] = bq + kth_bit(mq, k);
                else if (bq & kHubList) ev[u] = a.hlist[(bq & ~kHubList) + k];
                else ev[u] = bq + k;
            }
#pragma unroll
            for (int u = 0; u < kLsP; ++u) {
                iv[u] = 0; mfv[u] = 0; dsv[u] = 0; tfv[u] = 0; xq[u] = 0; rem[u] = false;
                xbk[u] = ~0ull; xbv[u] = 0;
                if (vv[u]) {
                    const uint32_t e = ev[u];
                    const int64_t pe = pv[u] + e;
                    iv[u] = a.col[e]; dsv[u] = a.dstate[e];
                    if (!mk[u]) mfv[u] = a.mflags[pe];
                    // a shard's push: a ghost receiver's records
                    // live on its own shard; the copy is a bit of its cross edge
                    rem[u] = a.push && (iv[u] < a.rlo || iv[u] >= a.rhi);
                    if (rem[u]) xq[u] = a.xwq[e];
                    else tfv[u] = a.tflags[pe];
                }
            }
            uint32_t clw = 0;
#pragma unroll
            for (int u = 0; u < kLsP; ++u) {
                if (!vv[u]) continue;
                const uint32_t j = jv[u], e = ev[u], i = iv[u], q = qv[u];
                const uint32_t m = s_m[q];
                const int32_t t = (int32_t)a.mtopic[m];
                const uint32_t origin = a.morigin[m];
                const ctp_t tp = const_tp(a.tp) + t;
                const uint8_t vd = a.minv[m];
                const bool inv = vd != GSIM_VERDICT_ACCEPT;
                const bool pen = verdict_penalises(vd), seeable = vd != GSIM_VERDICT_SIGNATURE;
                const uint8_t ds = dsv[u], tf = tfv[u];
                bool sel;
                if (mk[u]) {
                    sel = !(ds & GSIM_DS_DIRECT) || (a.mflags[pv[u] + e] & GSIM_TF_MESH);
                } else {
                    const uint8_t ow = (origin < a.N && ((a.sub[origin] >> t) & 1ull)) ? GSIM_TF_MESH : GSIM_TF_FANOUT;
                    sel = (mfv[u] & (j == origin ? ow : GSIM_TF_MESH)) != 0;
                }
                if (a.flood && j == origin) sel = ((a.sub[i] >> t) & 1ull) && a.score[a.rev[e]] >= a.pub_thr;
                if ((ds & GSIM_DS_DIRECT) && !sel) sel = (a.sub[i] >> t) & 1ull;
                const bool tg = sel && (ds & GSIM_DS_CONNECTED) && i != s_from[q] && i != origin;
                if (tg && rem[u]) {                  // the receiver's shard delivers it (k_xbits_deliver)
                    xbk[u] = (uint64_t)((int64_t)m * a.xbw + (xq[u] >> 6));
                    xbv[u] = 1ull << (xq[u] & 63u);
                    continue;
                }
                const bool ok = tg && (ds & GSIM_DS_ACCEPT);
                n_gray += tg && !ok;
                if (!ok) continue;
                if (a.subdyn && !((a.sub[i] >> t) & 1ull)) continue;   // a topic the receiver left
                n_acc++;
                const int64_t window = tp->mesh_message_deliveries_window_ns;
                const bool sc = tp->scored && (ds & GSIM_DS_TRACKED);
                const bool sbit = (a.seenbm[(int64_t)m * a.nw + (i >> 6)] >> (i & 63)) & 1ull;
                const bool wa = window >= 0 && a.now - round_time(a, a.mpub[m]) <= window;
                const bool known = sbit && (wa || !sc || inv || !(tf & GSIM_TF_IN_MESH));
                const int64_t ci = known ? 0 : a.cs.at((int64_t)a.cs.cbase[m], t, i);
                if (ci < 0) continue;
                uint32_t lo_w = j;
                if (sc && !inv) {
                    lo_w |= kCreditFirst;
                    if (window < 0 && (tf & GSIM_TF_IN_MESH)) lo_w |= kCreditMesh;
                }
                const uint64_t cv = ((uint64_t)(claim_hi | e) << 32) | lo_w;
                const bool fold = !sbit && seeable;
                const uint64_t c = known ? 0ull
                                 : fold ? __hip_atomic_fetch_min(a.cs.cell + ci, cv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                        : a.cs.cell[ci];
                const uint32_t chi = (uint32_t)(c >> 32);
                int64_t seen_round = -1;
                if (known) seen_round = a.g - 1;
                else if (c != kUnseen64) {
                    if (!(chi & kClaim)) seen_round = chi;
                    else if (((chi >> 30) & 1u) != (uint32_t)par) seen_round = a.g - 1;
                }
                if (fold || (seeable && seen_round < 0 && (c == kUnseen64 || (chi & kEdgeMask) > e))) {
                    const uint64_t prev = fold ? c
                                               : __hip_atomic_fetch_min(a.cs.cell + ci, cv, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_AGENT);
                    if (prev == kUnseen64) {
                        n_first++;
                        atomicOr(&s_new2[m >> 5], 1u << (m & 31));
                        clw |= 1u << u;
                        s_cl[u * kLsB + tid] = cl_entry(a, i, m, ci, (int64_t)a.cs.cbase[m]);
                    }
                }
                if (!sc) continue;
                const int64_t ir = pv[u] + e;
                if (pen) {
                    atomicAdd(&a.invalid[ir], 1.0);                   // markInvalidMessageDelivery
                    inv_mark(a);
                } else if (!inv && (tf & GSIM_TF_IN_MESH)) {
                    const bool in_window = known ? true
                                         : seen_round >= 0 ? (a.now - round_time(a, seen_round) <= window)
                                                           : (window >= 0);
                    if (in_window)
                        atomic_mcnt_inc(a.mcnt, ir, &a.meshd[ir], tp->mesh_message_deliveries_cap, a.mcnt_fast);
                }
            }
            if (a.push) {
#pragma unroll
                for (int u = 0; u < kLsP; ++u) xbits_or_wave(a.xbits, xbk[u], xbv[u]);
            }
            if (a.clist) {
#pragma unroll
                for (int u = 0; u < kLsP; ++u) clist_push_wave(a, (clw >> u) & 1u, s_cl[u * kLsB + tid]);
            }
        }
        __syncthreads();                                     // the entry tables are rewritten next
    }
    n_acc = wave_sum_u64(n_acc);
    n_gray = wave_sum_u64(n_gray);
    n_first = wave_sum_u64(n_first);
    if (lane == 0 && (n_acc | n_gray)) {
        atomicAdd(&s_stats[0], n_acc);
        atomicAdd(&s_stats[1], n_first);
        atomicAdd(&s_stats[3], n_gray);
    }
    __syncthreads();
    for (int w = tid; w < (a.ring + 31) / 32; w += kLsB) {
        uint32_t bits = s_new2[w];
        if (!bits) continue;
        slots_claimed(a, w, bits);
    }
    if (tid == 0 && (s_stats[0] | s_stats[3])) {
        stats_add(a, s_stats[0], s_stats[1], s_stats[3]);
    }
}

// A list the send round will not walk (the configuration changed since its
// commit; only_bad: the list is incomplete -- an entry did not fit, the device
// decides): its forwarders as fresh bits for k_send_tm.
__global__ __launch_bounds__(256) void k_flist_fresh(RoundArgs a, int only_bad)
{
    const int par = (int)(a.g & 1);
    if (only_bad && !a.fst[kFstBad + par]) return;       // complete: k_send_list walks it
    const int64_t n = min((int64_t)a.fst[par * kFstStride], a.flist_cap);
    const uint64_t* fl = a.flist + (int64_t)par * a.flist_cap;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = fl[k];
        const uint32_t x = fl_x(a, v), m = fl_m(a, v);
        fresh_set(a, m, (int64_t)(x >> 6), 1ull << (x & 63));
    }
}

// Copies that arrive as a list of (record, slot): round 2's messages queued by
// handleIWant (a shard's copies pushed by other shards arrive as bits:
// k_xbits_deliver).  Same rules and tracer events as k_send_tm's copies.
__global__ __launch_bounds__(256) void k_gossip_deliver(RoundArgs a_, const uint64_t* resp, const uint32_t* nresp,
                                                       const uint32_t* owner, int64_t resp_cap)
{
    const RoundArgs& a = a_;
    extern __shared__ uint32_t s_new2[];
    __shared__ unsigned long long s_stats[4];
    for (int w = threadIdx.x; w < (a.ring + 31) / 32; w += blockDim.x) s_new2[w] = 0;
    if (threadIdx.x < 4) s_stats[threadIdx.x] = 0;
    __syncthreads();
    // responses beyond the queue's capacity were dropped (reported as an
    // overflow by gsim_msg_stats): only the stored ones are read
    const uint32_t n = (uint32_t)min((int64_t)*nresp, resp_cap);
    const uint32_t par = (uint32_t)(a.g & 1);
    const uint32_t claim_hi = kClaim | (par << 30);
    const ctp_t tpa = const_tp(a.tp);
    unsigned long long n_acc = 0, n_gray = 0, n_first = 0;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
        const RoundArgs& a = kernarg0(a_);   // (re-read per copy: SGPR pressure)
        const uint64_t ent = resp[x];
        const uint32_t r = (uint32_t)ent, m = (uint32_t)(ent >> 32);
        if (a.tr.ev) {
            // the IWANT answer's RPC (a single engine: every entry is one), sent by
            // handleIWant in the round before it arrives (trace.go:250-297)
            const uint32_t rp = a.col[r], rs = owner[r];
            const int32_t rt = (int32_t)a.mtopic[m];
            // (a ghost advertiser's answers are known only at the requester's shard)
            if (a.tr.on_any(rs)) a.tr.push(round_time(a, a.g - 1), ((uint64_t)a.g << 32) | m, rs, rp, rt, GSIM_TRACE_SEND_RPC, 1);
            if (a.tr.on(rp)) a.tr.push(round_time(a, a.g), ((uint64_t)a.g << 32) | m, rp, rs, rt, GSIM_TRACE_RECV_RPC, 1);
        }
        listed_copy(a, r, m, owner, par, claim_hi, tpa, n_acc, n_gray, n_first, s_new2, true);
    }
    n_acc = wave_sum_u64(n_acc);
    n_gray = wave_sum_u64(n_gray);
    n_first = wave_sum_u64(n_first);
    if ((threadIdx.x & 63) == 0 && (n_acc | n_gray)) {
        atomicAdd(&s_stats[0], n_acc);
        atomicAdd(&s_stats[1], n_first);
        atomicAdd(&s_stats[3], n_gray);
    }
    __syncthreads();
    for (int w = threadIdx.x; w < (a.ring + 31) / 32; w += blockDim.x) {
        uint32_t bits = s_new2[w];
        if (!bits) continue;
        slots_claimed(a, w, bits);
    }
    if (threadIdx.x == 0 && (s_stats[0] | s_stats[3])) {
        stats_add(a, s_stats[0], s_stats[1], s_stats[3]);
    }
}

// applyIwantPenalties: the promises of ring index q expired before this
// heartbeat; a promise is broken unless its receiver has seen the message
// (fulfillPromise at first reception).  Record order: the penalty lands on
// the promiser's record of the advertiser, rev[e].
__global__ __launch_bounds__(256) void k_promise_check(uint32_t* prom_q, Cells cs, const uint32_t* mtopic,
                                                       const uint32_t* owner, const uint32_t* rev, uint8_t* pen,
                                                       int64_t E, unsigned long long* gstats)
{
    // promises sit at the promiser's (an owned receiver's) edges only
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long broken = 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) {
        const uint32_t slot = prom_q[e];
        if (slot == 0xFFFFFFFFu) continue;
        prom_q[e] = 0xFFFFFFFFu;
        if (cs.get(slot, (int32_t)mtopic[slot], owner[e]) == kUnseen64) {
            pen[rev[e]] = (uint8_t)(pen[rev[e]] + 1);
            ++broken;
        }
    }
    broken = wave_sum_u64(broken);
    if ((threadIdx.x & 63) == 0 && broken) atomicAdd(&gstats[3], broken);
}

// Start of round g: the validations completing now credit or penalise the
// copies queued for them (vq_push): the winner's markFirstMessageDelivery
// (its P2 from k_commit's kVqFirst, its P3 from its copy's kVqDup, as for
// the pending peers), the pending peers' markDuplicateMessageDelivery with validated zero (P3 if
// the record is in the mesh now, no window), RejectMessage's
// markInvalidMessageDelivery — each only if the record still exists
// (score.go:702-793, 901-981).  Every update is a capped +1 (or +1), so the
// queue order does not matter.
__global__ __launch_bounds__(256) void k_vq_apply(RoundArgs a, int pl)
{
    const int64_t scap = a.vq_cap / kVqSub;
    const int sub = (int)blockIdx.y;                       // one sub-list per grid row
    const uint64_t* q = a.vq + (int64_t)pl * a.vq_cap + sub * scap;
    const int64_t n = min((int64_t)a.vqn[vq_ctr(pl, sub)], scap);
    const ctp_t tpa = const_tp(a.tp);
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = q[x];
        const uint32_t e = (uint32_t)v, kind = (uint32_t)(v >> 40);
        const int32_t t = (int32_t)((v >> 32) & 0xFFu);
        if (!(a.dstate[e] & GSIM_DS_TRACKED)) continue;
        const uint64_t mj = smask_of(a.smask, a.owner[e]);     // the sender's row
        if (!slot_has(mj, t)) continue;
        const int64_t ir = slot_idx(mj, t, a.E, e);
        if (kind == kVqInv) { atomicAdd(&a.invalid[ir], 1.0); inv_mark(a); continue; }
        const ctp_t tp = tpa + t;
        // the winner's own copy was queued as kVqDup too: its kVqFirst adds
        // only markFirstMessageDelivery's P2 part
        if (kind == kVqFirst) atomic_inc_capped(&a.first[ir], tp->first_message_deliveries_cap);
        else if (a.tflags[ir] & GSIM_TF_IN_MESH) atomic_inc_capped(&a.meshd[ir], tp->mesh_message_deliveries_cap);
    }
}

// The counted pending copies of completion plane pl (dense layout, Deliver::
// d_vpc): per record, its invalid deliveries (markInvalidMessageDelivery, one
// +1 each) and, if in the mesh now, its duplicates (meshMessageDeliveries +1
// capped each) — the same +1 steps k_vq_apply makes for queue entries; the
// counts are cleared.  One thread per 8 records.
__global__ __launch_bounds__(256) void k_vq_counts(RoundArgs a, int pl)
{
    uint64_t* dw = reinterpret_cast<uint64_t*>(a.vpc + (int64_t)pl * a.vpe);
    uint64_t* iw = reinterpret_cast<uint64_t*>(a.vpc + (int64_t)(kVqPlanes + pl) * a.vpe);
    const int64_t nw = a.vpe >> 3;
    const ctp_t tpa = const_tp(a.tp);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
        const uint64_t dv = dw[w], iv = iw[w];
        if (!(dv | iv)) continue;
        dw[w] = 0;
        iw[w] = 0;
        for (int b = 0; b < 8; ++b) {
            const uint32_t nd = (uint32_t)(dv >> (8 * b)) & 0xFFu, ni = (uint32_t)(iv >> (8 * b)) & 0xFFu;
            if (!(nd | ni)) continue;
            const int64_t ir = w * 8 + b;
            const int32_t t = (int32_t)(ir / a.E);
            const int64_t e = ir - (int64_t)t * a.E;
            if (!(a.dstate[e] & GSIM_DS_TRACKED)) continue;
            if (ni) {
                double x = a.invalid[ir];
                for (uint32_t k = 0; k < ni; ++k) x = x + 1.0;
                a.invalid[ir] = x;
                inv_mark(a);
            }
            if (nd && (a.tflags[ir] & GSIM_TF_IN_MESH))
                a.meshd[ir] = apply_incs(a.meshd[ir], nd, (tpa + t)->mesh_message_deliveries_cap);
        }
    }
}

// End of round g: the cells whose validation completed in round g (claimed
// in round g - L of a slot with latency L, committed with hi = g) put the
// message in their mcache and, if accepted, forward it in round g + 1.
// hist: the slots with new claims of each round (Deliver::d_hist).
__global__ __launch_bounds__(256) void k_vcomplete(RoundArgs a, const uint32_t* hist, int32_t words)
{
    extern __shared__ uint16_t s_act[];
    __shared__ int s_n;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        int n = 0;
        for (int m0 = 0; m0 < a.ring; m0 += 64) {
            const int m = m0 + lane;
            const uint32_t L = m < a.ring ? a.mlat[m] : 0u;
            const bool act = L && a.g >= (int64_t)L &&
                             ((hist[(int64_t)((a.g - L) & (kVqPlanes - 1)) * words + (m >> 5)] >> (m & 31)) & 1u);
            const uint64_t b = __ballot(act);
            if (act) s_act[n + __popcll(b & ((1ull << lane) - 1))] = (uint16_t)m;
            n += __popcll(b);
        }
        if (lane == 0) s_n = n;
    }
    __syncthreads();
    const int nact = s_n;
    const int lane = threadIdx.x & 63;
    const int64_t i0 = ((int64_t)a.rlo & ~63ll) + ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
    if (i0 >= (int64_t)a.rhi || nact == 0) return;
    const int64_t i = i0 + lane;
    const bool vi = i < a.CN;
    const int32_t tick = (int32_t)(a.g / a.R);
    for (int k = 0; k < nact; ++k) {
        const uint32_t m = s_act[k];
        const int64_t ci = vi ? word_cell<true>(a.cs, a.mtopic, m, i0 >> 6, lane) : -1;
        const uint64_t c = ci >= 0 ? a.cs.cell[ci] : kUnseen64;
        const bool done = c != kUnseen64 && !((uint32_t)(c >> 32) & kClaim) && (int64_t)(c >> 32) == a.g;
        const uint64_t b = __ballot(done);
        if (!b) continue;
        const bool acc = a.minv[m] == GSIM_VERDICT_ACCEPT;
        if (done && acc) {                                // mcache.Put (this thread's peer alone)
            int32_t* lp = a.lastput + (int64_t)a.mtopic[m] * a.N + i;
            if (*lp < tick) *lp = tick;
        }
        if (lane == 0) {
            // slot-wide flags: every wave with a completion would hit the same
            // word; an atomic only while it still lacks the value
            if (__hip_atomic_load(&a.slot_last[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (int32_t)a.g)
                atomicMax(&a.slot_last[m], (int32_t)a.g);
            if (acc) {
                atomicOr(reinterpret_cast<unsigned long long*>(a.fresh + (int64_t)m * a.nw + (i0 >> 6)), b);
                atomicOr(reinterpret_cast<unsigned long long*>(a.fsum + (int64_t)m * a.nsw + (i0 >> 12)),
                         1ull << ((i0 >> 6) & 63));
                uint32_t* nn = a.nnew_cur + (m >> 5);
                if (!((__hip_atomic_load(nn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (m & 31)) & 1u))
                    atomicOr(nn, 1u << (m & 31));        // round g + 1 walks the slot
            }
        }
    }
}

// F_SEEN view [ring][N]: first-seen rounds of the peers with cells, unseen elsewhere
__global__ void k_seen_view(Cells cs, const uint32_t* mtopic, uint32_t* out, int64_t n, int64_t N)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += stride) {
        const int64_t m = x / N, i = x - m * N;
        out[x] = (uint32_t)(cs.get((uint32_t)m, (int32_t)mtopic[m], (uint32_t)i) >> 32);
    }
}

}  // namespace gsim

using namespace gsim;

// ---------------------------------------------------------------------------
// host side

static void dl_free(Deliver* d)
{
    if (!d) return;
    auto f = [](void* p) { if (p) (void)hipFree(p); };
    f(d->d_mtopic); f(d->d_morigin); f(d->d_minv); f(d->d_mid); f(d->d_cell); f(d->d_seenbm); f(d->d_fresh); f(d->d_fsum); f(d->d_mmask); f(d->d_tmtab); f(d->d_flist); f(d->d_fst); f(d->d_clist); f(d->d_clist_n); f(d->d_hidx); f(d->d_hrow); f(d->d_hlist); f(d->d_mlist); f(d->d_mloff); f(d->d_mcount); f(d->d_mmtab); f(d->d_hubw); f(d->d_mctab); f(d->d_ihm); f(d->d_mmb); f(d->d_mpub); f(d->d_roff); f(d->d_lastput);
    f(d->d_nnew); f(d->d_stats); f(d->d_seen32); f(d->d_pub);
    f(d->d_slot_last); f(d->d_gsel); f(d->d_gcount); f(d->d_gstate); f(d->d_resp); f(d->d_nresp); f(d->d_peertx); f(d->d_prom); f(d->d_pcand);
    f(d->d_behaviour); f(d->d_gstats);
    f(d->d_mlat); f(d->d_vq); f(d->d_vqn); f(d->d_hist); f(d->d_vpc);
    f(d->d_cbase); f(d->d_mbits); f(d->d_mpre); f(d->d_pslot); f(d->d_sched); f(d->d_sslot);
    delete d;
}

void free_deliver(gsim_handle* h)
{
    if (!h->dl) return;
    dl_free(h->dl);
    h->dl = nullptr;
}

bool deliver_field_ref(gsim_handle* h, int32_t f, gsim::FieldRef* r)
{
    Deliver* d = h->dl;
    if (!d) return false;
    if (f == GSIM_F_SEEN) { *r = {d->d_cell, (size_t)d->cfg.ring * (size_t)h->n * 4, FK_SEEN, 4}; return true; }
    if (f == GSIM_F_LASTPUT) { *r = {d->d_lastput, (size_t)std::max(1, h->t) * (size_t)h->n * 4}; return true; }
    return false;
}

static int nnew_words(const Deliver* d) { return (d->cfg.ring + 31) / 32; }

static int grid_peers(int64_t n)
{
    const int64_t waves = (n + 63) / 64;
    return (int)std::max<int64_t>((waves + 3) / 4, 1);
}


// Topic slots or member-compacted cells in use: the kernels' table-reading
// instances (SP = true); a dense layout runs the ones that index directly.
static bool sparse_layout(const gsim_handle* h)
{
    return h->d_smask != nullptr || (h->dl && h->dl->sparse != 0);
}

bool deliver_latency_on(gsim_handle* h) { return h->dl && h->dl->lat_on; }

// Member-major IHAVE passes: member lists of a sub-ring layout (a shard's
// members include its ghosts: their ghost rows hold their gossip marks into
// the shard, their cells the holdings their shards exported)
static bool mm_gossip(const gsim_handle* h)
{
    return h->dl && h->dl->d_mmtab && h->dl->sparse != 0;
}

// Commits from the claim list: member-compacted cells (sub-rings of topics
// only some peers hold) and no validation latency
static bool list_commit(const gsim_handle* h)
{
    return h->dl && h->dl->d_clist && h->dl->sparse != 0 && !h->dl->lat_on;
}

// The list-driven send (k_send_list) runs for this configuration: claim-list
// commits, and nothing k_send_list leaves to k_send_tm (the peer gater, the
// trace, the shards' pull exchange, validation latency)
static bool flist_allowed(const gsim_handle* h)
{
    return list_commit(h) && h->dl->d_flist && !h->gt && !h->trace.ev && (!h->sh || h->sh->push) && !h->flist_off;
}

static Cells deliver_cells(const Deliver* d)
{
    Cells c;
    c.cell = d->d_cell;
    c.cbase = d->d_cbase;
    c.mbits = d->d_mbits;
    c.mpre = d->d_mpre;
    c.nw = d->cell_nw;
    c.n = d->cell_nw ? d->n_peers : 0;
    c.sparse = d->sparse;
    return c;
}

static RoundArgs make_round_args(gsim_handle* h, int64_t g)
{
    Deliver* d = h->dl;
    RoundArgs a{};
    a.N = h->n; a.E = h->e; a.T = h->t; a.ring = d->cfg.ring; a.R = d->cfg.rounds;
    a.t0 = d->cfg.t0_ns; a.hb = d->cfg.heartbeat_ns; a.g = g;
    a.now = a.t0 + (g / a.R) * a.hb + (g % a.R + 1) * a.hb / (a.R + 1);
    a.row_ptr = h->d_row_ptr; a.col = h->d_col;
    a.dstate = h->d_dstate; a.mflags = h->d_mflags;
    a.smask = h->d_smask; a.owner = h->d_owner;
    a.tflags = h->d_tflags; a.tp = h->d_tp;
    a.first = h->d_first; a.meshd = h->d_meshd; a.invalid = h->d_invalid; a.mcnt = h->d_mcnt;
    a.mtopic = d->d_mtopic; a.morigin = d->d_morigin; a.minv = d->d_minv; a.mid = d->d_mid;
    a.mlat = d->lat_on ? d->d_mlat : nullptr;
    a.mlat_w = d->d_mlat;
    a.vq = d->d_vq; a.vqn = d->d_vqn; a.vq_cap = d->vq_cap;
    a.vpc = d->d_vpc; a.vpe = d->d_vpc ? (((int64_t)std::max(1, h->t) * h->e + 7) & ~(int64_t)7) : 0;
    a.cs = deliver_cells(d); a.lastput = d->d_lastput;
    a.CN = h->n;
    a.rlo = (uint32_t)h->olo();
    a.rhi = (uint32_t)h->ohi();
    a.seenbm = d->d_seenbm; a.nw = (a.CN + 63) / 64; a.mpub = d->d_mpub; a.roff = d->d_roff;
    a.fresh = d->d_fresh;
    a.fsum = d->d_fsum;
    a.mmask = d->d_mmask;
    a.hidx = d->d_hlist ? d->d_hidx : nullptr;
    a.hlist = d->d_hlist;
    a.tmtab = d->d_tmtab;
    a.peertx = d->d_peertx; a.ptx_w = d->ptx_w;
    a.tr = h->trace;
    a.nsw = (a.nw + 63) / 64;
    a.ncells = (int64_t)d->n_cells;
    a.gt = gater_ref(h);
    a.subdyn = h->sub_dynamic ? 1 : 0;
    if (a.gt.act) { a.gt.prom = d->d_prom; a.gt.P = d->prom_ticks; }
    a.topic_slots = d->cfg.topic_slots > 0 ? (int32_t)d->cfg.topic_slots : 0;
    if (list_commit(h)) {
        a.clist = d->d_clist;
        a.clist_n = d->d_clist_n;
        a.clist_cap = d->clist_cap;
        a.cl_j = GSIM_CL_PACK && h->n < (int64_t)kClPeerMax && d->cfg.ring <= kMaxRing ? 1 : 0;
    }
    if (flist_allowed(h)) {
        a.flist = d->d_flist;
        a.fst = d->d_fst;
        a.flist_cap = d->flist_cap;
        a.fl_from = GSIM_FL_PACK && h->n < (int64_t)kFlNone && d->cfg.ring <= kMaxRing ? 1 : 0;
    }
    const size_t w = (size_t)nnew_words(d);
    a.nnew_prev = d->d_nnew + (size_t)((g + 1) & 1) * w;
    a.nnew_cur = d->d_nnew + (size_t)(g & 1) * w;
    a.stats = d->d_stats;
    a.inv_live = h->d_inv_live ? h->d_inv_live + (h->inv_par & 1) : nullptr;
    a.slot_last = d->d_slot_last;
    a.err = d->d_nresp;
    a.reuse_guard = (std::max(h->gp.history_gossip, h->gp.history_length) + d->prom_ticks + 2) * d->cfg.rounds;
    a.mcnt_fast = !a.mlat && d->pub_bound > 0 && d->pub_bound < INT32_MAX &&
                  (int64_t)d->pub_bound * (1 + std::max(0, h->gp.gossip_retransmission)) <= 200;
    a.sub = h->d_sub; a.score = h->d_score; a.rev = h->d_rev;
    a.flood = h->gp.flood_publish ? 1 : 0;
    a.pub_thr = h->th.publish_threshold;
    a.slo = 0;
    a.shi = a.CN;
    if (ShardCtx* sh = h->sh) {
        a.sharded = 1;
        a.pgate = sh->d_pgate;
        if (sh->push) {
            // owned senders walk their whole rows; ghosts never send here
            a.push = 1;
            a.xwq = sh->d_xwq; a.xbits = sh->d_xbits; a.xbw = sh->xbw;
            a.slo = (sh->own_lo / (2 * kPushTB)) * (2 * kPushTB);   // whole chunks of the push walk
            a.shi = sh->own_hi;
        } else {
            a.sptr = sh->d_sptr;
            a.sedge = sh->d_sedge;
        }
    }
    return a;
}

bool deliver_gossip_view(gsim_handle* h, GossipView* v)
{
    Deliver* d = h->dl;
    if (!d) return false;
    v->lastput = d->d_lastput;
    v->gsel = d->d_gsel;
    v->gstate = d->d_gstate;
    v->mmask = d->d_mmask;
    return true;
}

bool deliver_wire_view(gsim_handle* h, WireView* v)
{
    Deliver* d = h->dl;
    if (!d) return false;
    v->cells = deliver_cells(d);
    v->mtopic = d->d_mtopic; v->morigin = d->d_morigin; v->minv = d->d_minv; v->mid = d->d_mid;
    v->slot_last = d->d_slot_last;
    v->gsel = d->d_gsel;
    v->ring = d->cfg.ring; v->rounds = d->cfg.rounds;
    v->ihave_tick = d->ihave_tick;
    return true;
}

static int64_t round_time_host(const Deliver* d, int64_t g)
{
    const int64_t R = d->cfg.rounds, hb = d->cfg.heartbeat_ns;
    return d->cfg.t0_ns + (g / R) * hb + (g % R + 1) * hb / (R + 1);
}

// applyIwantPenalties before the heartbeat at `now`: every promise ring index
// whose promises expired (expire.Before(now)) is checked and emptied; the
// penalties reach bp in the refresh pass that follows (before scoring).
int deliver_promise_check(gsim_handle* h, int64_t now)
{
    Deliver* d = h->dl;
    if (!d) return GSIM_OK;
    for (int q = 0; q < d->prom_ticks; ++q) {
        const int64_t made = d->prom_made[(size_t)q];
        if (made < 0) continue;
        const int64_t expire = round_time_host(d, made * d->cfg.rounds) + h->gp.iwant_followup_time_ns;
        if (!(expire < now)) continue;
        hipLaunchKernelGGL(k_promise_check, dim3(std::min<int64_t>((h->e + 255) / 256, 16384)), dim3(256), 0,
                           h->stream, d->d_prom + (size_t)q * (size_t)h->e, deliver_cells(d),
                           (const uint32_t*)d->d_mtopic, (const uint32_t*)h->d_owner, (const uint32_t*)h->d_rev,
                           h->d_pen, h->e, d->d_gstats);
        d->prom_made[(size_t)q] = -1;
        int rc = hip_check(h, hipGetLastError(), "k_promise_check");
        if (rc) return rc;
    }
    return GSIM_OK;
}

// The heartbeat's emitGossip rewrites the gossip choices of every joined topic.
int deliver_heartbeat_begin(gsim_handle* h, uint64_t tick)
{
    Deliver* d = h->dl;
    if (!d) return GSIM_OK;
    d->ihave_tick = (int64_t)tick;
    return GSIM_OK;
}

// Control round 0: handleIHave (+ the advertisers' handleIWant) for the
// heartbeat's IHAVE marks.  Staged so a sharded network can reduce the
// per-slot counts and share the holders between the stages (shard.hip).
namespace gsim {
struct IhaveStage {
    IhArgs a{};
    size_t lds, lds_c;
    int grid;
};
}  // namespace gsim

// false: no IHAVE handling in this round
static bool ihave_prepare(gsim_handle* h, int64_t g, IhaveStage* st, int* rc)
{
    *rc = GSIM_OK;
    Deliver* d = h->dl;
    const int64_t tick = g / d->cfg.rounds;
    if (d->ihave_tick != tick) return false;
    d->ihave_tick = -1;
    if (h->gp.max_ihave_messages < 1 || h->gp.max_ihave_length < 1) return false;
    IhArgs& a = st->a;
    a = IhArgs{};
    a.N = h->n; a.E = h->e; a.T = h->t; a.ring = d->cfg.ring; a.R = d->cfg.rounds;
    a.g = g; a.tick = tick;
    a.lo_round = (int32_t)std::max<int64_t>((tick - h->gp.history_gossip) * d->cfg.rounds, 0);
    a.row_ptr = h->d_row_ptr; a.col = h->d_col; a.rev = h->d_rev; a.sub = h->d_sub; a.smask = h->d_smask;
    a.mtopic = d->d_mtopic; a.morigin = d->d_morigin; a.minv = d->d_minv;
    a.mlat = d->lat_on ? d->d_mlat : nullptr;
    a.cs = deliver_cells(d); a.slot_last = d->d_slot_last;
    a.gsel = d->d_gsel; a.gstate = d->d_gstate; a.behaviour = d->d_behaviour;
    a.pcand = d->d_pcand; a.prom = d->d_prom; a.P = d->prom_ticks;
    a.prom_idx = (int32_t)(tick % d->prom_ticks);
    if (d->prom_made[(size_t)a.prom_idx] >= 0) {
        h->err = "IWANT promise ring index still pending (refresh_scores must run every heartbeat)";
        *rc = GSIM_ESTATE;
        return false;
    }
    d->prom_made[(size_t)a.prom_idx] = tick;
    a.resp = d->d_resp; a.nresp = d->d_nresp; a.resp_cap = d->resp_cap; a.gstats = d->d_gstats;
    a.respond = h->gp.gossip_retransmission >= 1;
    a.seed = h->x ? gsim_get_seed(h) : 0;
    a.CN = h->n;
    a.rlo = (uint32_t)h->olo();
    a.rhi = (uint32_t)h->ohi();
    if (ShardCtx* sh = h->sh) {
        a.sharded = 1;
        a.gid = sh->d_gid;
    }
    a.max_ihave = h->gp.max_ihave_length;
    a.tr = h->trace;
    a.t0 = d->cfg.t0_ns; a.hb = d->cfg.heartbeat_ns; a.roff = d->d_roff;
    a.peertx = d->d_peertx; a.ptx_w = d->ptx_w;
    a.retrans = h->gp.gossip_retransmission;
    if (mm_gossip(h)) {
        a.mlist = d->d_mlist; a.mloff = d->d_mloff; a.mcount = d->d_mcount; a.mmtab = d->d_mmtab;
        a.topic_slots = (int32_t)d->cfg.topic_slots;
        a.ihm = d->d_ihm; a.mmb = d->d_mmb;
        // the hub-row list: at most every wave of the launch (grow-only)
        const int64_t need = 4 * (int64_t)(d->mmtab.empty() ? 0 : d->mmtab.back());
        if (need > d->hubw_cap) {
            if (d->d_hubw) { (void)hipFree(d->d_hubw); d->d_hubw = nullptr; d->hubw_cap = 0; }
            if (hipMalloc((void**)&d->d_hubw, sizeof(uint32_t) * (size_t)(need + 1)) == hipSuccess) d->hubw_cap = need;
        }
        if (d->d_hubw && need > 0) {
            a.hubw = d->d_hubw;
            a.hubn = d->d_hubw + d->hubw_cap;
        }
    }
    st->lds = (((size_t)d->cfg.ring + 3) & ~(size_t)3) * sizeof(uint16_t) + 4 * kRespStage * sizeof(uint64_t);
    st->lds_c = (((size_t)d->cfg.ring + 1) & ~(size_t)1) * sizeof(uint16_t) + 2 * (size_t)d->cfg.ring * 4;
    st->grid = grid_peers(a.CN);
    hipError_t e = hipMemsetAsync(d->d_nresp, 0, 2 * sizeof(uint32_t), h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_nresp + 3, 0, sizeof(uint32_t), h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_gcount, 0, 2 * (size_t)d->cfg.ring * 4, h->stream);
    if (e != hipSuccess) { *rc = hip_check(h, e, "gossip reset"); return false; }
    return true;
}

// Holders and wanting receivers per slot (d_gcount), over the peers with cells.
static int ihave_count(gsim_handle* h, IhaveStage* st)
{
    ProfScope ps(h, GSIM_K_GOSSIP);
    Deliver* d = h->dl;
    if (st->a.mmtab) {
        const uint32_t grid = d->mctab.back();
        const size_t lds = 2 * (size_t)d->cfg.topic_slots * 4;
        if (grid && st->a.mlat)
            hipLaunchKernelGGL(k_gossip_count_mm<true>, dim3(grid), dim3(256), lds, h->stream, st->a,
                               (const uint32_t*)d->d_mctab, d->d_gcount);
        else if (grid)
            hipLaunchKernelGGL(k_gossip_count_mm<false>, dim3(grid), dim3(256), lds, h->stream, st->a,
                               (const uint32_t*)d->d_mctab, d->d_gcount);
    } else if (st->a.mlat)
        hipLaunchKernelGGL((k_gossip_count<true, true>), dim3(st->grid), dim3(256), st->lds_c, h->stream, st->a, h->dl->d_gcount);
    else if (sparse_layout(h))
        hipLaunchKernelGGL((k_gossip_count<false, true>), dim3(st->grid), dim3(256), st->lds_c, h->stream, st->a, h->dl->d_gcount);
    else
        hipLaunchKernelGGL((k_gossip_count<false, false>), dim3(st->grid), dim3(256), st->lds_c, h->stream, st->a, h->dl->d_gcount);
    return hip_check(h, hipGetLastError(), "k_gossip_count");
}

template <int W>
static void launch_ihave_w(gsim_handle* h, IhaveStage* st, const IhArgs& a)
{
    if (a.mmtab) {
        const uint32_t grid = h->dl->mmtab.back();
        if (!grid) return;
        const uint32_t* gc = h->dl->d_gcount;
        if (a.hubw && W < 64) {
            // rows of at most kIhHub connections, listing the waves with longer ones;
            // then those rows, kIhSlices blocks of one wave per listed wave
            uint32_t n = 0;
            hipError_t e = hipMemsetAsync(a.hubn, 0, sizeof(uint32_t), h->stream);
            if (e != hipSuccess) return;
            if (a.mlat)
                hipLaunchKernelGGL((k_ihave<W, true, true, true, 1>), dim3(grid), dim3(256), st->lds, h->stream, a, gc);
            else
                hipLaunchKernelGGL((k_ihave<W, false, true, true, 1>), dim3(grid), dim3(256), st->lds, h->stream, a, gc);
            e = hipMemcpyAsync(&n, a.hubn, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
            if (e != hipSuccess || n == 0) return;
            const uint32_t g2 = n * (uint32_t)kIhSlices;
            if (a.mlat)
                hipLaunchKernelGGL((k_ihave<W, true, true, true, 2>), dim3(g2), dim3(64), st->lds, h->stream, a, gc);
            else
                hipLaunchKernelGGL((k_ihave<W, false, true, true, 2>), dim3(g2), dim3(64), st->lds, h->stream, a, gc);
            return;
        }
        if (a.mlat)
            hipLaunchKernelGGL((k_ihave<W, true, true, true>), dim3(grid), dim3(256), st->lds, h->stream, a, gc);
        else
            hipLaunchKernelGGL((k_ihave<W, false, true, true>), dim3(grid), dim3(256), st->lds, h->stream, a, gc);
    } else if (a.mlat)
        hipLaunchKernelGGL((k_ihave<W, true, true>), dim3(st->grid), dim3(256), st->lds, h->stream, a, (const uint32_t*)h->dl->d_gcount);
    else if (sparse_layout(h))
        hipLaunchKernelGGL((k_ihave<W, false, true>), dim3(st->grid), dim3(256), st->lds, h->stream, a, (const uint32_t*)h->dl->d_gcount);
    else
        hipLaunchKernelGGL((k_ihave<W, false, false>), dim3(st->grid), dim3(256), st->lds, h->stream, a, (const uint32_t*)h->dl->d_gcount);
}

static int ihave_walk(gsim_handle* h, IhaveStage* st)
{
    Deliver* d = h->dl;
    IhArgs& a = st->a;
    ProfScope ps(h, GSIM_K_GOSSIP);
    // lane groups sized to the rows: power-law graphs (long rows, short mean) walk
    // their few long rows in chunks rather than idling 3/4 of a 64-lane group
    int w = h->ihave_w;
    if (w == 0) {
        const bool short_mean = h->e <= 24 * (int64_t)h->n;
        w = (h->max_degree <= 16 || (h->max_degree > 32 && short_mean)) ? 16 : h->max_degree <= 32 ? 32 : 64;
    }
    if (w == 8)
        launch_ihave_w<8>(h, st, a);
    else if (w == 16)
        launch_ihave_w<16>(h, st, a);
    else if (w == 32)
        launch_ihave_w<32>(h, st, a);
    else
        launch_ihave_w<64>(h, st, a);
    if (d->cfg.ring > h->gp.max_ihave_length) {
        // the window may hold more than MaxIHaveLength slots: k_gossip_count
        // decided on the device which of the two walks runs
        const size_t lds = (((size_t)d->cfg.ring + 3) & ~(size_t)3) * sizeof(uint16_t) +
                           4 * (kRespStage + kPairTopics) * sizeof(uint64_t) + 4 * kPairTopics * sizeof(uint32_t);
        const int grid = (int)std::min<int64_t>((a.CN + 3) / 4, 4096);
        if (a.mlat) hipLaunchKernelGGL(k_ihave_pairs<true>, dim3(grid), dim3(256), lds, h->stream, a);
        else hipLaunchKernelGGL(k_ihave_pairs<false>, dim3(grid), dim3(256), lds, h->stream, a);
    }
    hipLaunchKernelGGL(k_promise_insert, dim3(std::min<int64_t>((h->e + 255) / 256, 16384)), dim3(256), 0, h->stream,
                       d->d_pcand, d->d_prom, d->prom_ticks, a.prom_idx, h->e);
    d->resp_round = a.g + 2;
    return hip_check(h, hipGetLastError(), "k_ihave");
}

static int launch_ihave(gsim_handle* h, int64_t g)
{
    IhaveStage st;
    int rc = GSIM_OK;
    if (!ihave_prepare(h, g, &st, &rc)) return rc;
    rc = ihave_count(h, &st);
    if (!rc) rc = ihave_walk(h, &st);
    return rc;
}

int deliver_flush(gsim_handle* h)
{
    Deliver* d = h->dl;
    if (!d || d->pending < 0) return GSIM_OK;
    ProfScope ps(h, GSIM_K_COMMIT);
    RoundArgs a = make_round_args(h, d->pending);
    a.flist_commit = a.flist != nullptr;       // round g+1's forwarders go to its list, not the fresh bits
    d->flist_round = a.flist ? d->pending + 1 : -1;
    // member-compacted cells: a capped grid (the scan usually exits at once: the
    // claim list covers the round); dense: a wave per word
    const int gp = grid_peers((int64_t)a.rhi - ((int64_t)a.rlo & ~63ll));
    const dim3 grid(sparse_layout(h) ? std::min(gp, 8192) : gp);
    // a shard's few words (< 2^14, dense, no latency or gater): 4 slot groups
    // (the single engine's 15.6 k words at C3 keep a wave per word: split over 4 / 8
    // topic groups its commit took 5.43 / 6.03 against 4.47 ms per tick, gpurun_out/r05t_c3;
    // a slot batch's lastput / credit loads issued before its stores: 5.32,
    // gpurun_out/r05u_c3 -- not the claims' serial read-modify-writes, then)
    const bool split = gp < 4096 && h->sh && !a.mlat && !a.gt.act && !sparse_layout(h);
    if (a.clist)
        hipLaunchKernelGGL(k_commit_list<true>, dim3(64, kClSub), dim3(256), 0, h->stream, a);
    if (a.mlat)
        hipLaunchKernelGGL((k_commit<true, true>), grid, dim3(256), (size_t)d->cfg.ring * sizeof(uint16_t), h->stream, a);
    else if (a.gt.act && sparse_layout(h))
        hipLaunchKernelGGL((k_commit<false, true, true>), grid, dim3(256), (size_t)d->cfg.ring * sizeof(uint16_t), h->stream, a);
    else if (a.gt.act)
        hipLaunchKernelGGL((k_commit<false, false, true>), grid, dim3(256), (size_t)d->cfg.ring * sizeof(uint16_t), h->stream, a);
    else if (sparse_layout(h))
        hipLaunchKernelGGL((k_commit<false, true>), grid, dim3(256), (size_t)d->cfg.ring * sizeof(uint16_t), h->stream, a);
    else if (split)
        // (a wave per word: 4 words per wave were slower, profiles/r05_shards8_ab_ranges_split.txt)
        hipLaunchKernelGGL((k_commit<false, false, false, true>), dim3(gp, GSIM_SPLIT_GROUPS), dim3(256),
                           (size_t)d->cfg.ring * sizeof(uint16_t),
                           h->stream, a);
    else
        hipLaunchKernelGGL((k_commit<false, false>), grid, dim3(256), (size_t)d->cfg.ring * sizeof(uint16_t), h->stream, a);
    const int64_t committed = d->pending;
    d->pending = -1;
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && a.clist) e = hipMemsetAsync(d->d_clist_n, 0, (kClSub + 1) * kClStride * sizeof(uint32_t), h->stream);
    const int rc = hip_check(h, e, "k_commit");
    return rc ? rc : gater_fold(h, committed, a.now);    // the round's gater events, claims resolved
}

// The previous tick's IWANT response queue overflow and early slot reuse,
// checked at the heartbeat (one small synchronous read per tick) so a caller
// that never asks for gsim_msg_stats still stops before running on with
// state that has diverged.
static int vq_check(gsim_handle* h)
{
    Deliver* d = h->dl;
    if (!d->lat_on) return GSIM_OK;
    uint32_t ov = 0;
    hipError_t e = hipMemcpyAsync(&ov, d->d_vqn + kVqOver, sizeof(ov), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "validation queue flag");
    if (ov) { h->err = "copies pending validation overflowed their queue (raise gsim_msg_config.max_arrivals)"; return GSIM_ERANGE; }
    return GSIM_OK;
}

int deliver_check_errors(gsim_handle* h)
{
    Deliver* d = h->dl;
    if (!d) return GSIM_OK;
    if (int rc = vq_check(h)) return rc;
    uint32_t err[4] = {0, 0, 0, 0};
    hipError_t e = hipMemcpyAsync(err, d->d_nresp, sizeof(err), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "delivery error flags");
    if (err[1]) { h->err = "IWANT responses overflowed their queue (raise gsim_msg_config.max_arrivals)"; return GSIM_ERANGE; }
    if (err[2]) {
        h->err = "a ring slot was republished while its message could still be gossiped or promised (raise ring)";
        return GSIM_ESTATE;
    }
    return GSIM_OK;
}

bool deliver_trace_view(gsim_handle* h, TraceView* v)
{
    Deliver* d = h->dl;
    if (!d) return false;
    v->cells = deliver_cells(d); v->mtopic = d->d_mtopic; v->minv = d->d_minv; v->mid = d->d_mid;
    v->ring = d->cfg.ring; v->rounds = d->cfg.rounds;
    v->mlat = d->lat_on ? d->d_mlat : nullptr;
    v->t0 = d->cfg.t0_ns; v->hb = d->cfg.heartbeat_ns; v->roff = d->d_roff;
    return true;
}

int64_t deliver_last_round_time(gsim_handle* h)
{
    const Deliver* d = h->dl;
    if (!d || d->next_round <= 0) return INT64_MAX;
    return round_time_host(d, d->next_round - 1);
}

int deliver_read_seen(gsim_handle* h, void* dst)
{
    Deliver* d = h->dl;
    int rc = deliver_flush(h);
    if (rc) return rc;
    const size_t n = (size_t)d->cfg.ring * (size_t)h->n;
    hipError_t e = hipSuccess;
    if (!d->d_seen32) e = hipMalloc((void**)&d->d_seen32, std::max<size_t>(n * 4, 4));
    if (e != hipSuccess) return hip_check(h, e, "seen view scratch");
    hipLaunchKernelGGL(k_seen_view, dim3(std::min<int64_t>(((int64_t)n + 255) / 256, 16384)), dim3(256), 0, h->stream,
                       deliver_cells(d), (const uint32_t*)d->d_mtopic, d->d_seen32, (int64_t)n, h->n);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(dst, d->d_seen32, n * 4, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return hip_check(h, e, "gsim_read_field(SEEN)");
}

static int launch_send_tm(gsim_handle* h, const RoundArgs& a0)
{
    // blocks per topic: about 2048 blocks in all (8 per CU over the launch at one
    // resident block per CU: smaller ranges even out the frontier work; measured
    // 512 / 1024 / 1536 / 2048 / 3072 / 4096 blocks: 30.5 / 22.7 / 21.4 / 20.9 /
    // 21.1 / 21.3 ms per tick at C3, profiles/r01_ab_send_tm_blocks.log), ranges of
    // at least 4096 peers; at least 256 ranges per topic when there are many
    // topics (Zipf subscriptions skew them: the busy topics' blocks must still
    // fill the chip; blocks of idle topics leave after the slot scan).  c5 block
    // budgets 4096 / 8192 / 15680 (default) / 32768 / 65536: 29.7 / 25.0 / 24.7 /
    // 28.0 / 32.9 ms of send per tick (profiles/r02_ab_send_blocks.log)
    constexpr int TB = GSIM_TM_TB;
    const bool sp = sparse_layout(h);
    const int TBv = a0.push ? kPushTB : sp ? kSparseTB : TB;
    const int64_t total = 2048 * (1024 / TBv);
    const int64_t chunk = 2 * TBv;
    // every local peer sends (pull: a shard's ghosts too), or the owned range (push)
    const int64_t cn = a0.shi - a0.slo;
    const int T = std::max(1, h->t);
    // ranges down to one chunk: a small network (c2: 10k peers, one topic) still
    // spreads its frontier over several CUs (4096-peer ranges gave it 3 blocks:
    // 122 us of send per round); large ones are capped by the budget below
    // (a shard's push walk too: ranges of 2 / 4 chunks were slower,
    // profiles/r05_shards8_ab_ranges_split.txt)
    const int64_t min_range = chunk;
    const int64_t ranges = std::max<int64_t>(1, std::min<int64_t>((cn + min_range - 1) / min_range,
                                                                    std::max<int64_t>(h->t >= 32 ? 256 : 1,
                                                                                      total / T)));
    Deliver* d = h->dl;
    if (d->tm_cn != cn || d->tm_tb != TBv) {
        // the same budget of ranges x T blocks, shared out by subscribers
        // (Zipf topics: the busiest topic's blocks set the launch's length),
        // ranges of whole chunks
        int64_t wsum = 0;
        for (int t = 0; t < T && !h->tm_uniform; ++t) wsum += t < (int)h->topic_subs.size() ? h->topic_subs[t] : 0;
        const int64_t budget = h->tm_budget ? h->tm_budget : ranges * T, max_blocks = (cn + chunk - 1) / chunk;
        d->tmtab.assign((size_t)(2 * T + 1), 0);
        uint32_t start = 0;
        for (int t = 0; t < T; ++t) {
            int64_t b = ranges;
            if (wsum > 0) b = (budget * h->topic_subs[t] + wsum - 1) / wsum;
            // ranges of at most kMaxRange peers: a quiet topic's block still scans
            // its range chunk by chunk, and one block over all N peers would
            // set the launch's length
            const int64_t kMaxRange = 64 * chunk;
            b = std::max<int64_t>(std::max<int64_t>(1, (cn + kMaxRange - 1) / kMaxRange), std::min(b, max_blocks));
            const int64_t range = ((cn + b - 1) / b + chunk - 1) / chunk * chunk;
            d->tmtab[t] = start;
            d->tmtab[T + 1 + t] = (uint32_t)range;
            start += (uint32_t)((cn + range - 1) / range);
        }
        d->tmtab[T] = start;
        hipError_t e = hipMemcpyAsync(d->d_tmtab, d->tmtab.data(), d->tmtab.size() * 4, hipMemcpyHostToDevice,
                                      h->stream);
        if (e != hipSuccess) return hip_check(h, e, "k_send_tm block table");
        d->tm_cn = cn;
        d->tm_tb = TBv;
    }
    const RoundArgs& a = a0;
    // the slot list in LDS
    const size_t lds = ((size_t)d->cfg.ring * 2 + 7) & ~(size_t)7;
    const dim3 grid(d->tmtab[T]);
    if (a.push && a.mlat)
        hipLaunchKernelGGL((k_send_tm<kPushTB, true, true, false, true>), grid, dim3(kPushTB), lds,
                           h->stream, a);
    else if (a.push && a.gt.act && sp)
        hipLaunchKernelGGL((k_send_tm<kPushTB, false, true, true, true>), grid, dim3(kPushTB), lds,
                           h->stream, a);
    else if (a.push && a.gt.act)
        hipLaunchKernelGGL((k_send_tm<kPushTB, false, false, true, true>), grid, dim3(kPushTB), lds,
                           h->stream, a);
    else if (a.push && sp)
        hipLaunchKernelGGL((k_send_tm<kPushTB, false, true, false, true>), grid, dim3(kPushTB), lds,
                           h->stream, a);
    else if (a.push)
        hipLaunchKernelGGL((k_send_tm<kPushTB, false, false, false, true>), grid, dim3(kPushTB), lds,
                           h->stream, a);
    else if (a.mlat && sp)
        hipLaunchKernelGGL((k_send_tm<kSparseTB, true, true>), grid, dim3(kSparseTB), lds, h->stream, a);
    else if (a.mlat)
        hipLaunchKernelGGL((k_send_tm<TB, true, true>), grid, dim3(TB), lds, h->stream, a);
    else if (a.gt.act && sp)
        hipLaunchKernelGGL((k_send_tm<kSparseTB, false, true, true>), grid, dim3(kSparseTB), lds, h->stream, a);
    else if (a.gt.act)
        hipLaunchKernelGGL((k_send_tm<TB, false, false, true>), grid, dim3(TB), lds, h->stream, a);
    else if (sp)
        hipLaunchKernelGGL((k_send_tm<kSparseTB, false, true>), grid, dim3(kSparseTB), lds, h->stream, a);
    else
        hipLaunchKernelGGL((k_send_tm<TB, false, false>), grid, dim3(TB), lds, h->stream, a);
    return hip_check(h, hipGetLastError(), "k_send_tm");
}

// Round g's send: the forwarder list (k_send_list) when the commit of round
// g-1 left it complete, else the scan of the fresh bits (k_send_tm, which
// exits at once when the list covers the round: the device decides, the
// list may have overflowed)
static int launch_send(gsim_handle* h, RoundArgs& a, int64_t round)
{
    Deliver* d = h->dl;
    const bool listed = d->flist_round == round;
    const bool walk = listed && flist_allowed(h);
    d->flist_round = -1;
    if (listed && !walk && d->d_flist) {
        // the configuration changed since the commit: the list as fresh bits
        RoundArgs b = a;
        b.flist = d->d_flist; b.fst = d->d_fst; b.flist_cap = d->flist_cap;
        hipLaunchKernelGGL(k_flist_fresh, dim3(1024), dim3(256), 0, h->stream, b, 0);
    }
    if (walk)   // an overflowed list (device flag): its entries as fresh bits for the scan
        hipLaunchKernelGGL(k_flist_fresh, dim3(1024), dim3(256), 0, h->stream, a, 1);
    a.flist_send = walk ? 1 : 0;
    int rc = launch_send_tm(h, a);
    if (!rc && walk) {
        const size_t lds = (size_t)nnew_words(d) * 4;
        hipLaunchKernelGGL(k_send_list, dim3(2048), dim3(kLsB), lds, h->stream, a);
        rc = hip_check(h, hipGetLastError(), "k_send_list");
    }
    if (!rc && d->d_fst) {
        // this round's list is consumed: its parity is refilled by the next commit
        const int p = (int)(round & 1);
        hipError_t e = hipMemsetAsync(d->d_fst + p * kFstStride, 0, 4, h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(d->d_fst + kFstBad + p, 0, 4, h->stream);
        rc = hip_check(h, e, "forwarder list reset");
    }
    return rc;
}

// ---- round stages (gsim_round runs them in order; a sharded group
// exchanges copies between send and post, control records after control,
// and the IHAVE counts / holders inside the IHAVE stage, shard.hip) --------

static bool lazy_commits(const gsim_handle* h)
{
    // commits may trail their round only while every window is >= 0: with a
    // negative window the first delivery's P3 credit must land before control
    for (const auto& tp : h->tp)
        if (tp.scored && tp.mesh_message_deliveries_window_ns < 0) return false;
    return true;
}

// Stage 1 of round g: order checks, AcceptFrom verdicts of a new score
// snapshot, and (topic-major delivery) the commits of round g-1, which set
// the fresh bits of round g's forwarders.
int deliver_round_prepare(gsim_handle* h, int64_t round)
{
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    if (round < 0 || round >= 0x7FFFFFFF) { h->err = "round out of range [0, 2^31-1)"; return GSIM_ERANGE; }
    if (d->next_round >= 0 && round != d->next_round) {
        h->err = "rounds must be consecutive";
        return GSIM_ESTATE;
    }
    int rc = 0;
    {
        ProfScope ps(h, GSIM_K_ACCEPT);
        rc = refresh_accept(h);
        if (rc) return rc;
    }
    rc = deliver_flush(h);
    if (!rc && d->lat_on) {
        // validations completing now (the flush above queued round g-1's
        // winners with latency 1)
        ProfScope ps(h, GSIM_K_COMMIT);
        RoundArgs a = make_round_args(h, round);
        const int pl = (int)(round & (kVqPlanes - 1));
        hipLaunchKernelGGL(k_vq_apply, dim3(128, kVqSub), dim3(256), 0, h->stream, a, pl);
        if (d->d_vpc)
            hipLaunchKernelGGL(k_vq_counts, dim3((uint32_t)std::min<int64_t>((a.vpe / 8 + 255) / 256, 16384)), dim3(256),
                               0, h->stream, a, pl);
        hipError_t e = hipMemsetAsync(d->d_vqn + vq_ctr(pl, 0), 0, sizeof(uint32_t) * kVqSub * kVqStride, h->stream);
        if (e == hipSuccess) e = hipGetLastError();
        rc = hip_check(h, e, "k_vq_apply");
    }
    return rc;
}

// End of round g (validation latencies): the round's claims are recorded for
// their completion round, and the cells completing now put and forward.
int deliver_round_validate(gsim_handle* h, int64_t round)
{
    Deliver* d = h->dl;
    if (!d->lat_on) return GSIM_OK;
    ProfScope ps(h, GSIM_K_COMMIT);
    RoundArgs a = make_round_args(h, round);
    const int w = nnew_words(d);
    hipError_t e = hipMemcpyAsync(d->d_hist + (size_t)(round & (kVqPlanes - 1)) * (size_t)w, a.nnew_cur,
                                  (size_t)w * 4, hipMemcpyDeviceToDevice, h->stream);
    if (e != hipSuccess) return hip_check(h, e, "validation history");
    hipLaunchKernelGGL(k_vcomplete, dim3(grid_peers((int64_t)a.rhi - ((int64_t)a.rlo & ~63ll))), dim3(256),
                       (size_t)d->cfg.ring * sizeof(uint16_t), h->stream, a, (const uint32_t*)d->d_hist, w);
    return hip_check(h, hipGetLastError(), "k_vcomplete");
}

// Stage 2: the delivery kernel of round g.
static int xbits_gather(gsim_handle* h, int64_t round);   // (below: the copy bits)

int deliver_round_send(gsim_handle* h, int64_t round)
{
    Deliver* d = h->dl;
    int rc = 0;
    RoundArgs a = make_round_args(h, round);
    h->mcnt_dirty = true;
    // the receivers a forwarder's walk covers: every peer (push), else the owned ones
    const uint32_t mlo = a.push ? 0u : (uint32_t)h->olo(), mhi = a.push ? (uint32_t)h->n : (uint32_t)h->ohi();
    {
        ProfScope ps(h, GSIM_K_SEND);
        if (d->mask_version != h->mesh_version) {
            // the masks are kept current by the heartbeat, the control pass
            // and a shard's router import; other writers of the router's
            // flags (ABI writes, direct peers, the device fill) bump the
            // version: rebuild them all
            hipLaunchKernelGGL(k_mesh_mask, dim3((uint32_t)std::min<int64_t>((h->n + 3) / 4, 65536)), dim3(256), 0,
                               h->stream, (const uint32_t*)h->d_row_ptr, (const uint32_t*)h->d_col,
                               (const uint8_t*)h->d_mflags, (const uint8_t*)h->d_direct,
                               (const uint64_t*)h->d_smask, h->n, h->e,
                               std::max(1, h->t), mlo, mhi, d->d_mmask,
                               a.push ? h->olo() : (int64_t)0, a.push ? h->ohi() : h->n);   // push: owned senders only
            d->mask_version = h->mesh_version;
            d->hub_round = -1;
        }
        // hub lists: after the heartbeat (round 0 of a tick) and the control
        // rounds (0, 1) and any rebuild of the masks
        if (d->d_hlist && (d->hub_round < 0 || round % d->cfg.rounds < 3)) {
            hipLaunchKernelGGL(k_hub_mesh, dim3((uint32_t)std::min<int64_t>((d->nhub + 3) / 4, 65536)), dim3(256), 0,
                               h->stream, (const uint32_t*)h->d_row_ptr, (const uint32_t*)h->d_col,
                               (const uint8_t*)h->d_mflags, (const uint8_t*)h->d_direct,
                               (const uint64_t*)h->d_smask, (const uint32_t*)d->d_hrow, d->nhub, h->e,
                               std::max(1, h->t), mlo, mhi, d->d_hlist);
            d->hub_round = round;
        }
        // one thread per edge: forwarders walk only their mesh edges (a
        // handful of a row's positions), so lane groups per row would idle
        // most lanes (C3: 21.0 against 32.9 ms per tick,
        // profiles/r02_ab_walk_masks.log)
        rc = gater_round_begin(h, a.now);   // the gate's state before the round's copies
        if (!rc) rc = launch_send(h, a, round);
        if (rc) return rc;
        gater_round_sent(h, round);
        if (h->sh && h->sh->push) {                    // the copies to ghost receivers, per destination
            rc = xbits_gather(h, round);
            if (rc) return rc;
        }
        // the claims of round g-1 were committed before k_send_tm; round g+1's bits
        // were last read (as "previous") by round g
        d->pending = round;
        hipError_t e = hipMemsetAsync(d->d_nnew + (size_t)((round + 1) & 1) * (size_t)nnew_words(d), 0,
                                      (size_t)nnew_words(d) * 4, h->stream);
        if (e != hipSuccess) return hip_check(h, e, "nnew reset");
    }
    return hip_check(h, hipGetLastError(), "k_send");
}

// Copies arriving in round g at this handle's peers, one entry per copy:
// the receiver's record of the sender | slot << 32 (the IWANT responses).
// *d_n entries, at most cap.
int deliver_round_queue(gsim_handle* h, int64_t round, const uint64_t* q, const uint32_t* d_n, int64_t cap)
{
    Deliver* d = h->dl;
    RoundArgs a = make_round_args(h, round);
    const size_t lds2 = (size_t)nnew_words(d) * 4;
    hipLaunchKernelGGL(k_gossip_deliver, dim3(2048), dim3(256), lds2, h->stream, a, q, d_n,
                       (const uint32_t*)h->d_owner, cap);
    return hip_check(h, hipGetLastError(), "k_gossip_deliver");
}

// ---- copy push as bitmaps -------------------------------
// A round's copies to ghost receivers are bits of xbits ([ring][xbw] words,
// k_send_tm<PUSH>).  The gather lists each destination's segment of every
// active slot (the slots k_send_tm walked: nnew_prev), slot ids first, and
// clears it:  out[d] = [m_0 .. m_{n-1}] [n x xw_d words]; cnt[0] = n.
__global__ __launch_bounds__(256) void k_xbits_gather(const uint32_t* nnew, int32_t ring, uint64_t* xbits, int64_t xbw,
                                                      const int64_t* xwo, uint64_t* out, int64_t out_cap, uint32_t* cnt)
{
    extern __shared__ uint16_t s_act[];
    __shared__ int s_n;
    const int n = active_slots(nnew, ring, s_act, &s_n);
    const int d = (int)blockIdx.y;
    const int64_t w0 = xwo[d], xw = xwo[d + 1] - w0;
    uint64_t* o = out + (int64_t)d * out_cap;
    if (blockIdx.x == 0) {
        for (int k = threadIdx.x; k < n && xw > 0; k += blockDim.x) o[k] = s_act[k];
        if (d == 0 && threadIdx.x == 0) *cnt = (uint32_t)n;
    }
    const int64_t tot = (int64_t)n * xw;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < tot; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = x / xw, w = x - k * xw;
        uint64_t* src = xbits + (int64_t)s_act[k] * xbw + w0 + w;
        const uint64_t v = *src;
        o[n + x] = v;
        if (v) *src = 0;
    }
}

// The bits from every other shard: per source q, n slots of xw words, a bit
// at position b of slot m's words is a copy of m on record gbase + b (the
// ghost block of q's peers, in q's cross-out order).  A wave takes 64 words
// of one slot and applies their copies in record order (the set bits listed
// in LDS), so neighbouring lanes touch neighbouring records.
constexpr int kXbList = 1024;                // per-wave LDS list of a task's copies

// waves per SIMD the bit apply is fitted to: 6 (80 VGPRs, no spill) against 5
// (94): mean shard 11.66 / 11.67 -> 11.56 / 11.61 ms (gpurun_out/r05h_ab); two
// copies per lane in flight (kXbP) against four: 11.82 / 11.76
#ifndef GSIM_XB_WPE
#define GSIM_XB_WPE 6
#endif

// listed_copy for kXbP copies of slot m per lane at once (records rr[], ~0u:
// none), the common configuration only -- dense cells, no claim list, topic
// slots, gater, trace, Leave or validation latency (xbits_fast) -- with the
// same rules and results; each stage's loads for all the copies are issued
// before any is used, so the copies' dependent trips overlap.
#ifndef GSIM_XB_P
#define GSIM_XB_P 2
#endif
constexpr int kXbP = GSIM_XB_P;
__device__ __forceinline__ void listed_copies_fast(const RoundArgs& a, const uint32_t* rr, uint32_t m, int32_t t,
                                                   const uint32_t* owner, uint32_t claim_hi, uint32_t par, ctp_t tp,
                                                   unsigned long long& n_acc, unsigned long long& n_gray,
                                                   unsigned long long& n_first, uint32_t* s_new2)
{
    const uint8_t vd = a.minv[m];
    const bool inv = vd != GSIM_VERDICT_ACCEPT, pen = verdict_penalises(vd);
    const int64_t window = tp->mesh_message_deliveries_window_ns;
    const double mcap = tp->mesh_message_deliveries_cap;
    bool on[kXbP], sc[kXbP], known[kXbP];
    uint8_t ds[kXbP], tf[kXbP];
    uint32_t p[kXbP];
    uint64_t sw[kXbP], c[kXbP];
#pragma unroll
    for (int u = 0; u < kXbP; ++u) {                     // stage 1: the record's edge state
        on[u] = rr[u] != ~0u;
        ds[u] = on[u] ? a.dstate[rr[u]] : 0;
        p[u] = on[u] ? a.col[rr[u]] : 0u;
        tf[u] = on[u] ? a.tflags[(int64_t)t * a.E + rr[u]] : 0;
    }
#pragma unroll
    for (int u = 0; u < kXbP; ++u) {                     // AcceptFrom; stage 2: the committed bit
        if (on[u] && !(ds[u] & GSIM_DS_ACCEPT)) { n_gray++; on[u] = false; }
        n_acc += on[u];
        sc[u] = on[u] && tp->scored && (ds[u] & GSIM_DS_TRACKED);
        sw[u] = on[u] ? a.seenbm[(int64_t)m * a.nw + (p[u] >> 6)] : 0ull;
    }
    const bool wa = window >= 0 && a.now - round_time(a, a.mpub[m]) <= window;
#pragma unroll
    for (int u = 0; u < kXbP; ++u) {                     // stage 3: the cells that matter
        const bool sb = (sw[u] >> (p[u] & 63)) & 1ull;
        known[u] = on[u] && sb && (wa || !sc[u] || inv || !(tf[u] & GSIM_TF_IN_MESH));
        c[u] = (on[u] && !known[u]) ? a.cs.cell[(int64_t)m * a.cs.n + p[u]] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kXbP; ++u) {
        if (!on[u]) continue;
        const uint32_t r = rr[u];
        const int64_t ir = (int64_t)t * a.E + r;
        int64_t seen_round = -1;
        if (!known[u]) {
            const uint32_t hi = (uint32_t)(c[u] >> 32);
            if (c[u] != kUnseen64) {
                if (!(hi & kClaim)) seen_round = hi;
                else if (((hi >> 30) & 1u) != par) seen_round = a.g - 1;
            }
            if (vd != GSIM_VERDICT_SIGNATURE && seen_round < 0 && (c[u] == kUnseen64 || (hi & kEdgeMask) > r)) {
                uint32_t lo = owner[r];
                if (sc[u] && !inv) {
                    lo |= kCreditFirst;
                    if (window < 0 && (tf[u] & GSIM_TF_IN_MESH)) lo |= kCreditMesh;
                }
                const uint64_t v = ((uint64_t)(claim_hi | r) << 32) | lo;
                const uint64_t prev = __hip_atomic_fetch_min(a.cs.cell + (int64_t)m * a.cs.n + p[u], v, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
                if (prev == kUnseen64) {
                    n_first++;
                    atomicOr(&s_new2[m >> 5], 1u << (m & 31));
                }
            }
        }
        if (!sc[u]) continue;
        if (pen) {
            atomicAdd(&a.invalid[ir], 1.0);                           // markInvalidMessageDelivery
            inv_mark(a);
        } else if (!inv && (tf[u] & GSIM_TF_IN_MESH)) {
            const bool in_window = known[u] ? true
                                 : seen_round >= 0 ? (a.now - round_time(a, seen_round) <= window) : (window >= 0);
            if (in_window) atomic_mcnt_inc(a.mcnt, ir, &a.meshd[ir], mcap, a.mcnt_fast);
        }
    }
}
__global__ __launch_bounds__(256, GSIM_XB_WPE) void k_xbits_deliver(RoundArgs a_, const uint64_t* in, const XSrc* src, int32_t K,
                                                       int64_t ntask, const uint32_t* owner, int32_t xbits_fast_on)
{
    const RoundArgs& a = a_;
    extern __shared__ uint32_t s_new2[];
    __shared__ uint32_t s_list[4][kXbList];
    __shared__ unsigned long long s_stats[4];
    for (int w = threadIdx.x; w < (a.ring + 31) / 32; w += blockDim.x) s_new2[w] = 0;
    if (threadIdx.x < 4) s_stats[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t par = (uint32_t)(a.g & 1);
    const uint32_t claim_hi = kClaim | (par << 30);
    const ctp_t tpa = const_tp(a.tp);
    unsigned long long n_acc = 0, n_gray = 0, n_first = 0;
    uint32_t* lst = s_list[wid];
    // the common configuration: listed_copies_fast (kXbP copies per lane in flight)
    const bool fast = !a.smask && !a.cs.sparse && !a.clist && !a.gt.act && !a.tr.ev && !a.subdyn && !a.mlat &&
                      xbits_fast_on;
    for (int64_t tk = (int64_t)blockIdx.x * 4 + wid; tk < ntask; tk += (int64_t)gridDim.x * 4) {   // wave-uniform
        const RoundArgs& a = kernarg0(a_);
        int q = 0;
        while (q + 1 < K && src[q + 1].toff <= tk) ++q;
        const XSrc sq = src[q];
        const int64_t cpw = ((int64_t)sq.xw + 63) / 64;
        const int64_t rel = tk - sq.toff, k = rel / cpw, c0 = (rel - k * cpw) * 64;
        const uint32_t m = (uint32_t)in[sq.in_off + k];
        const int64_t w = c0 + lane;
        const uint64_t bits = w < sq.xw ? in[sq.in_off + sq.n + k * sq.xw + w] : 0ull;
        const uint32_t cnt = (uint32_t)__popcll(bits);
        uint32_t pre = cnt;                                   // inclusive scan over the wave
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)pre, o, 64);
            if (lane >= o) pre += y;
        }
        const uint32_t total = (uint32_t)__shfl((int)pre, 63, 64);
        if (!total) continue;
        const int64_t rb = sq.gbase + w * 64;
        if (total <= (uint32_t)kXbList) {
            uint32_t pos = pre - cnt;
            for (uint64_t b = bits; b; b &= b - 1) lst[pos++] = (uint32_t)(w * 64) + (uint32_t)__builtin_ctzll(b);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            if (fast) {
                const int32_t t = (int32_t)a.mtopic[m];
                for (uint32_t j0 = 0; j0 < total; j0 += 64 * kXbP) {
                    uint32_t rr[kXbP];
#pragma unroll
                    for (int u = 0; u < kXbP; ++u) {
                        const uint32_t j = j0 + (uint32_t)(u * 64 + lane);
                        rr[u] = j < total ? (uint32_t)(sq.gbase + lst[j]) : ~0u;
                    }
                    listed_copies_fast(a, rr, m, t, owner, claim_hi, par, tpa + t, n_acc, n_gray, n_first, s_new2);
                }
            } else {
                for (uint32_t j0 = 0; j0 < total; j0 += 64) {
                    if (j0 + lane < total)
                        listed_copy(a, (uint32_t)(sq.gbase + lst[j0 + lane]), m, owner, par, claim_hi, tpa, n_acc, n_gray,
                                    n_first, s_new2, false);
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   // lst is rewritten by the next task
        } else {
            for (uint64_t b = bits; b; b &= b - 1)
                listed_copy(a, (uint32_t)(rb + __builtin_ctzll(b)), m, owner, par, claim_hi, tpa, n_acc, n_gray, n_first,
                            s_new2, false);
        }
    }
    n_acc = wave_sum_u64(n_acc);
    n_gray = wave_sum_u64(n_gray);
    n_first = wave_sum_u64(n_first);
    if (lane == 0 && (n_acc | n_gray)) {
        atomicAdd(&s_stats[0], n_acc);
        atomicAdd(&s_stats[1], n_first);
        atomicAdd(&s_stats[3], n_gray);
    }
    __syncthreads();
    for (int w = threadIdx.x; w < (a.ring + 31) / 32; w += blockDim.x) {
        uint32_t bits = s_new2[w];
        if (!bits) continue;
        slots_claimed(a, w, bits);
    }
    if (threadIdx.x == 0 && (s_stats[0] | s_stats[3])) {
        stats_add(a, s_stats[0], s_stats[1], s_stats[3]);
    }
}

// right after round g's k_send_tm, while its slots (nnew of g-1) are still set
static int xbits_gather(gsim_handle* h, int64_t round)
{
    Deliver* d = h->dl;
    ShardCtx* sh = h->sh;
    hipLaunchKernelGGL(k_xbits_gather, dim3(64, (uint32_t)sh->K), dim3(256), (size_t)d->cfg.ring * sizeof(uint16_t),
                       h->stream, (const uint32_t*)(d->d_nnew + (size_t)((round + 1) & 1) * (size_t)nnew_words(d)),
                       d->cfg.ring, sh->d_xbits, sh->xbw, (const int64_t*)sh->d_xwo, sh->d_xsend, sh->xsend_cap, sh->d_xn);
    return hip_check(h, hipGetLastError(), "k_xbits_gather");
}

int deliver_xbits_apply(gsim_handle* h, int64_t round, const uint64_t* in, const XSrc* d_src, int K, int64_t ntask)
{
    if (ntask <= 0) return GSIM_OK;
    Deliver* d = h->dl;
    RoundArgs a = make_round_args(h, round);
    const size_t lds2 = (size_t)nnew_words(d) * 4;
    // (blocks that fill the chip several times over: each block's end-of-run
    // slot and total updates contend on a few addresses)
    const uint32_t grid = (uint32_t)std::min<int64_t>((ntask + 3) / 4, 2048);
    hipLaunchKernelGGL(k_xbits_deliver, dim3(grid), dim3(256), lds2, h->stream, a, in, d_src, (int32_t)K,
                       ntask, (const uint32_t*)h->d_owner, (int32_t)(h->xb_generic ? 0 : 1));
    return hip_check(h, hipGetLastError(), "k_xbits_deliver");
}

// the pending meshd increments were applied (refresh, materialize_mcnt)
void deliver_mcnt_applied(gsim_handle* h)
{
    Deliver* d = h->dl;
    if (d && d->next_round >= 0) d->applied_tick = d->next_round / std::max(1, d->cfg.rounds);
}

int deliver_round_post(gsim_handle* h, int64_t round)
{
    Deliver* d = h->dl;
    int rc = GSIM_OK;
    if (d->resp_round == round) {
        // the messages handleIWant sent in control round 1 arrive with this round's copies
        ProfScope ps(h, GSIM_K_GOSSIP);
        rc = deliver_round_queue(h, round, d->d_resp, d->d_nresp, d->resp_cap);
        d->resp_round = -1;
        if (rc) return rc;
    }
    if (!lazy_commits(h)) rc = deliver_flush(h);
    return rc;
}

int deliver_round_control(gsim_handle* h, int64_t round)
{
    Deliver* d = h->dl;
    const int32_t r = (int32_t)(round % d->cfg.rounds);
    // rounds >= 2 of a heartbeat have an empty control inbox: handling PRUNE
    // replies (round 1) emits nothing
    if (r >= 2) return GSIM_OK;
    RoundArgs a = make_round_args(h, round);
    return handle_control(h, r, a.now);
}

int deliver_round_ihave(gsim_handle* h, int64_t round)
{
    return round % h->dl->cfg.rounds == 0 ? launch_ihave(h, round) : GSIM_OK;
}

void deliver_round_end(gsim_handle* h, int64_t round) { h->dl->next_round = round + 1; }

// ---- a sharded network's frontier exchange -----------------
// Round g's forwarders among a shard's owned peers (their fresh bits, set by
// the commits of round g-1 and by publication), one entry each: global peer
// id | global id of its first sender << 24 (0xFFFFFF: none) | slot << 48.
// Every other shard imports the entries of its ghosts: the ghost's cell gets
// the first-seen round and first sender, its fresh bit and the slot's
// activity are set, so that shard's k_send_tm walks the ghost's row (its
// connections into the shard) and delivers those copies itself.
constexpr uint64_t kG24 = 0xFFFFFFull;

// One thread per (active slot, owned word); a block's entries are written
// in item order (slot-major, ascending peers: the importers' cell and bitmap
// writes coalesce) at a range reserved with one atomic.
__global__ __launch_bounds__(256) void k_frontier_export(RoundArgs a, const uint32_t* gid, uint64_t* out, uint32_t* cnt,
                                                         int64_t cap)
{
    extern __shared__ uint16_t s_act[];
    __shared__ int s_n;
    __shared__ uint32_t s_wsum[4], s_base;
    const int nact = active_slots(a.nnew_prev, a.ring, s_act, &s_n);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t w0 = (int64_t)a.rlo >> 6, nwd = (((int64_t)a.rhi + 63) >> 6) - w0;
    const int64_t items = nwd * nact;
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < items; b0 += (int64_t)gridDim.x * 256) {   // block-uniform
        const int64_t x = b0 + tid;
        uint64_t bits = 0;
        uint32_t m = 0;
        int64_t w = 0;
        if (x < items) {
            const int64_t k = x / nwd;
            w = w0 + (x - k * nwd);
            m = s_act[k];
            bits = a.fresh[(int64_t)m * a.nw + w];
            if (w * 64 < (int64_t)a.rlo) bits &= ~0ull << ((int64_t)a.rlo - w * 64);        // owned peers only
            if (w * 64 + 64 > (int64_t)a.rhi) bits &= (1ull << ((int64_t)a.rhi - w * 64)) - 1;
        }
        const uint32_t c = (uint32_t)__popcll(bits);
        uint32_t v = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)v, o, 64);
            if (lane >= o) v += y;
        }
        if (lane == 63) s_wsum[wid] = v;
        __syncthreads();
        if (tid == 0) {
            const uint32_t tot = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
            s_wsum[3] = s_wsum[0] + s_wsum[1] + s_wsum[2];
            s_wsum[2] = s_wsum[0] + s_wsum[1];
            s_wsum[1] = s_wsum[0];
            s_wsum[0] = 0;
            s_base = tot ? atomicAdd(cnt, tot) : 0u;
        }
        __syncthreads();
        int64_t pos = (int64_t)s_base + s_wsum[wid] + (v - c);
        for (uint64_t b = bits; b; b &= b - 1, ++pos) {
            const int64_t i = w * 64 + __ffsll((long long)b) - 1;
            const uint64_t c = a.cs.get(m, (int32_t)a.mtopic[m], (uint32_t)i);
            const uint32_t f = (uint32_t)c & kPeerMask;
            // push: the cell's first-seen (or validation-completion) round in
            // place of the first sender, which no other shard reads
            const uint64_t gf = a.push ? ((c >> 32) & kG24) : f < a.N ? (uint64_t)gid[f] : kG24;
            if (pos < cap) out[pos] = (uint64_t)gid[i] | (gf << 24) | ((uint64_t)m << 48);
        }
        __syncthreads();
    }
}

// The ghosts among the other shards' forwarders.  Entries come in runs of
// one slot and ascending peers: the summary and activity bits are touched
// once per run.
__global__ __launch_bounds__(256) void k_frontier_import(RoundArgs a, const uint32_t* g2l, const uint64_t* in,
                                                         int64_t n)
{
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t b0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); b0 < n; b0 += stride) {   // wave-uniform
        const int64_t x = b0 + lane;
        bool ghost = false, fwd = false;
        uint32_t l = 0, m = 0;
        if (x < n) {
            const uint64_t v = in[x];
            l = g2l[v & kG24];
            ghost = l != 0xFFFFFFFFu && !(l >= a.rlo && l < a.rhi);         // a ghost of this shard
            if (ghost) {
                // (push: only the round is read, by IHAVE, and comes with the
                // entry; pull: the first sender too, by the ghost's walk)
                const uint64_t gf = a.push ? kG24 : (v >> 24) & kG24;
                uint32_t f = gf == kG24 ? 0xFFFFFFFFu : g2l[gf];
                if (f == 0xFFFFFFFFu) f = kPeerMask;                         // not a local peer
                const uint32_t fr = a.push ? (uint32_t)((v >> 24) & kG24) : (uint32_t)(a.g - 1);
                m = (uint32_t)(v >> 48);
                const int64_t ci = a.cs.idx(m, (int32_t)a.mtopic[m], l);    // a forwarder holds the topic
                if (ci >= 0) a.cs.cell[ci] = ((uint64_t)fr << 32) | f;
                // (filtering out ghosts without mesh edges into this shard, by
                // their masks, cost more in the import than it saved in the
                // walk: K = 8 serial shards 31.8 against 20.2 ms per tick)
                // push: the cell alone (IHAVE holders); the ghost's own shard sends
                fwd = !a.push;
            }
        }
        // one atomic per run of equal (slot, word) keys: a segmented OR scan
        // over the wave (the entries come sorted by slot and peer, so equal
        // keys are contiguous); the run's last lane holds its bits
        const uint64_t kw = fwd ? (uint64_t)m * (uint64_t)a.nw + (l >> 6) : ~0ull;
        uint64_t bits = fwd ? 1ull << (l & 63) : 0ull;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t ko = (uint64_t)__shfl_up((long long)kw, o, 64);
            const uint64_t vo = (uint64_t)__shfl_up((long long)bits, o, 64);
            if (lane >= o && ko == kw) bits |= vo;
        }
        const uint64_t kn = (uint64_t)__shfl_down((long long)kw, 1, 64);
        if (fwd && (lane == 63 || kn != kw)) {
            atomicOr(reinterpret_cast<unsigned long long*>(a.fresh + kw), bits);
            const int64_t w = (int64_t)(l >> 6);
            atomicOr(reinterpret_cast<unsigned long long*>(a.fsum + (int64_t)m * a.nsw + (w >> 6)), 1ull << (w & 63));
        }
        // the slot's activity: forwarding next round (nnew), mcache (slot_last)
        const uint32_t mn = (uint32_t)__shfl_down((int)(ghost ? m : 0xFFFFFFFFu), 1, 64);
        const uint32_t fwn = (uint32_t)__shfl_down((int)(fwd ? m : 0xFFFFFFFFu), 1, 64);
        if (fwd && (lane == 63 || fwn != m)) {
            uint32_t* nw = const_cast<uint32_t*>(a.nnew_prev) + (m >> 5);
            if (!((__hip_atomic_load(nw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (m & 31)) & 1u))
                atomicOr(nw, 1u << (m & 31));
        }
        // (push: the entries of a tick carry their own rounds; pull: all g - 1)
        if (ghost && (a.push || lane == 63 || mn != m)) {
            const int32_t fr = a.push ? (int32_t)(uint32_t)((in[x] >> 24) & kG24) : (int32_t)(a.g - 1);
            if (__hip_atomic_load(&a.slot_last[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < fr)
                atomicMax(&a.slot_last[m], fr);
        }
    }
}

// Push: a ghost's cell is read by IHAVE only, against the
// gossip window's tick-aligned bounds, so the holders go out once per tick as
// bits.  Each round ORs its forwarders (fresh bits of the round's slots) into
// the bitmap of the tick of their first-seen round (a publication's origin
// belongs to the round's own tick, every other forwarder to the round
// before's), over global words of the owned range.
__global__ __launch_bounds__(256) void k_holder_accum(RoundArgs a, uint64_t* hb, uint32_t* hs, int64_t how, int64_t gw0,
                                                      int64_t glo, int64_t ghi)
{
    extern __shared__ uint16_t s_act[];
    __shared__ int s_n;
    const int64_t hw = (int64_t)((a.ring + 31) / 32);
    uint32_t* s_hs = reinterpret_cast<uint32_t*>(s_act + ((a.ring + 1) & ~1));   // [2][hw] the slots touched
    for (int64_t w = threadIdx.x; w < 2 * hw; w += blockDim.x) s_hs[w] = 0;
    const int nact = active_slots(a.nnew_prev, a.ring, s_act, &s_n);
    const int64_t items = (int64_t)nact * how;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < items; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = x / how, w = x - k * how;
        const uint32_t m = s_act[k];
        const int64_t gp0 = (gw0 + w) * 64;                // global peer of bit 0
        const int64_t lb = (int64_t)a.rlo + (gp0 - glo);    // its local bit (glo: a multiple of 64)
        const uint64_t* f = a.fresh + (int64_t)m * a.nw;
        uint64_t bits = 0;
        if (lb >= 0) {
            const int64_t lw = lb >> 6;
            const int sh = (int)(lb & 63);
            bits = f[lw] >> sh;
            if (sh && lw + 1 < a.nw) bits |= f[lw + 1] << (64 - sh);
        }
        if (gp0 + 64 > ghi) bits &= ghi - gp0 >= 64 ? ~0ull : ((1ull << (ghi - gp0)) - 1ull);   // owned peers only
        if (!bits) continue;
        // forwarders of round g first saw the message in round g-1, or in g (a
        // publication's origin): only the first round of a tick tells them apart
        // (with validation latencies the cells say: a completion round)
        uint64_t mp[2] = {0, 0};
        const int pg = (int)((a.g / a.R) & 1);
        if (a.g % a.R != 0 && !a.mlat) {
            mp[pg] = bits;
        } else {
            const int32_t t = (int32_t)a.mtopic[m];
            for (uint64_t b = bits; b; b &= b - 1) {
                const int q = __builtin_ctzll(b);
                const uint64_t c = a.cs.get(m, t, (uint32_t)(lb + q));
                const int64_t fr = (int64_t)((c >> 32) & kG24);
                mp[(fr / a.R) & 1] |= 1ull << q;
            }
        }
        for (int p = 0; p < 2; ++p) {
            if (!mp[p]) continue;
            hb[((int64_t)p * a.ring + m) * how + w] |= mp[p];
            atomicOr(&s_hs[p * hw + (m >> 5)], 1u << (m & 31));   // (one global atomic per block and word, below)
        }
    }
    __syncthreads();
    for (int64_t w = threadIdx.x; w < 2 * hw; w += blockDim.x)
        if (s_hs[w]) atomicOr(&hs[w], s_hs[w]);
}

// The tick's holder bits (parity p): the slots touched, then their words,
// cleared as they are read; *cnt = the slots.
__global__ __launch_bounds__(256) void k_holder_gather(uint64_t* hb, const uint32_t* hs, int32_t ring, int64_t how,
                                                       uint64_t* out, uint32_t* cnt)
{
    extern __shared__ uint16_t s_act[];
    __shared__ int s_n;
    const int n = active_slots(hs, ring, s_act, &s_n);
    if (blockIdx.x == 0) {
        for (int k = threadIdx.x; k < n; k += blockDim.x) out[k] = s_act[k];
        if (threadIdx.x == 0) *cnt = (uint32_t)n;
    }
    const int64_t tot = (int64_t)n * how;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < tot; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = x / how, w = x - k * how;
        uint64_t* src = hb + (int64_t)s_act[k] * how + w;
        const uint64_t v = *src;
        out[n + x] = v;
        if (v) *src = 0;
    }
}

// Every other shard's holders of tick k: each set bit that is a ghost here
// gets its cell (first-seen round fr, the tick's first; no local sender) and
// the slot's activity.  A wave takes 64 words of one (source, slot).
__global__ __launch_bounds__(256) void k_holder_import(RoundArgs a, const uint32_t* g2l, const uint64_t* in,
                                                       const HSrc* src, int32_t K, int64_t ntask, int64_t fr)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int64_t tk = (int64_t)blockIdx.x * 4 + wid; tk < ntask; tk += (int64_t)gridDim.x * 4) {   // wave-uniform
        int q = 0;
        while (q + 1 < K && src[q + 1].toff <= tk) ++q;
        const HSrc sq = src[q];
        const int64_t cpw = ((int64_t)sq.nw + 63) / 64;
        const int64_t rel = tk - sq.toff, k = rel / cpw, w0 = (rel - k * cpw) * 64;
        const uint32_t m = (uint32_t)in[sq.in_off + k];
        const int32_t t = (int32_t)a.mtopic[m];
        const uint64_t mine = w0 + lane < sq.nw ? in[sq.in_off + sq.n + k * sq.nw + w0 + lane] : 0ull;
        // word by word, lane b taking bit b: the peers' g2l entries and cells
        // are consecutive (most holders' words are dense); kHiP words at a time,
        // their g2l loads issued before any cell store (one trip, not kHiP)
        constexpr int kHiP = 4;
        for (uint64_t wm = __ballot(mine != 0); wm;) {
            int jv[kHiP];
            uint32_t lv[kHiP];
#pragma unroll
            for (int u = 0; u < kHiP; ++u) {                                // wave-uniform
                jv[u] = wm ? __builtin_ctzll(wm) : -1;
                if (wm) wm &= wm - 1;
            }
#pragma unroll
            for (int u = 0; u < kHiP; ++u) {
                const uint64_t bits = jv[u] >= 0 ? (uint64_t)__shfl((long long)mine, jv[u], 64) : 0ull;
                lv[u] = ((bits >> lane) & 1ull) ? g2l[sq.pbase + (w0 + jv[u]) * 64 + lane] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int u = 0; u < kHiP; ++u) {
                const uint32_t l = lv[u];
                if (l == 0xFFFFFFFFu || (l >= a.rlo && l < a.rhi)) continue;  // not a ghost of this shard
                const int64_t ci = a.cs.idx(m, t, l);                          // a forwarder holds the topic
                if (ci >= 0) a.cs.cell[ci] = ((uint64_t)fr << 32) | kPeerMask;
            }
        }
        if (__ballot(mine != 0) && lane == 0 &&
            __hip_atomic_load(&a.slot_last[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (int32_t)fr)
            atomicMax(&a.slot_last[m], (int32_t)fr);
    }
}

int deliver_holder_accum(gsim_handle* h, int64_t round)
{
    if (round == 0) return GSIM_OK;
    Deliver* d = h->dl;
    ShardCtx* sh = h->sh;
    RoundArgs a = make_round_args(h, round);
    const int64_t gw0 = sh->bounds[(size_t)sh->k] >> 6;
    const int64_t items = sh->how * (int64_t)d->cfg.ring;   // an upper bound: the active slots are on the device
    const size_t lds = (size_t)((d->cfg.ring + 1) & ~1) * sizeof(uint16_t) + 2 * (size_t)((d->cfg.ring + 31) / 32) * 4;
    hipLaunchKernelGGL(k_holder_accum, dim3((uint32_t)std::max<int64_t>(1, std::min<int64_t>((items + 255) / 256, 1024))),
                       dim3(256), lds, h->stream, a, sh->d_hbits, sh->d_hslots,
                       sh->how, gw0, (int64_t)sh->bounds[(size_t)sh->k], (int64_t)sh->bounds[(size_t)sh->k + 1]);
    return hip_check(h, hipGetLastError(), "k_holder_accum");
}

int deliver_holder_gather(gsim_handle* h, int parity)
{
    Deliver* d = h->dl;
    ShardCtx* sh = h->sh;
    const int64_t hw = (d->cfg.ring + 31) / 32;
    hipLaunchKernelGGL(k_holder_gather, dim3(256), dim3(256), (size_t)d->cfg.ring * sizeof(uint16_t), h->stream,
                       sh->d_hbits + (size_t)parity * (size_t)d->cfg.ring * (size_t)sh->how,
                       (const uint32_t*)(sh->d_hslots + (size_t)parity * (size_t)hw), d->cfg.ring, sh->how, sh->d_hsend,
                       sh->d_hn);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemsetAsync(sh->d_hslots + (size_t)parity * (size_t)hw, 0, (size_t)hw * 4, h->stream);
    return hip_check(h, e, "k_holder_gather");
}

int deliver_holder_import(gsim_handle* h, int64_t round, const uint64_t* in, const HSrc* d_src, int K, int64_t ntask,
                          int64_t fr)
{
    if (ntask <= 0) return GSIM_OK;
    RoundArgs a = make_round_args(h, round);
    const uint32_t grid = (uint32_t)std::min<int64_t>((ntask + 3) / 4, 8192);
    hipLaunchKernelGGL(k_holder_import, dim3(grid), dim3(256), 0, h->stream, a, (const uint32_t*)h->sh->d_g2l, in, d_src,
                       (int32_t)K, ntask, fr);
    return hip_check(h, hipGetLastError(), "k_holder_import");
}

int deliver_frontier_export(gsim_handle* h, int64_t round, uint64_t* out, uint32_t* d_cnt, int64_t cap, bool append)
{
    Deliver* d = h->dl;
    RoundArgs a = make_round_args(h, round);
    if (!append) {
        hipError_t e = hipMemsetAsync(d_cnt, 0, sizeof(uint32_t), h->stream);
        if (e != hipSuccess) return hip_check(h, e, "frontier count");
    }
    if (round == 0) return GSIM_OK;
    const int64_t words = ((h->ohi() + 63) >> 6) - (h->olo() >> 6);
    const int64_t items = words * (int64_t)d->cfg.ring;      // an upper bound: the active slots are on the device
    hipLaunchKernelGGL(k_frontier_export, dim3((uint32_t)std::max<int64_t>(1, std::min<int64_t>((items + 255) / 256, 2048))),
                       dim3(256), (size_t)d->cfg.ring * sizeof(uint16_t), h->stream, a, (const uint32_t*)h->sh->d_gid,
                       out, d_cnt, cap);
    return hip_check(h, hipGetLastError(), "k_frontier_export");
}

int deliver_frontier_import(gsim_handle* h, int64_t round, const uint64_t* in, int64_t n)
{
    if (n <= 0 || round == 0) return GSIM_OK;
    RoundArgs a = make_round_args(h, round);
    hipLaunchKernelGGL(k_frontier_import, dim3((uint32_t)std::min<int64_t>((n + 255) / 256, 16384)), dim3(256), 0,
                       h->stream, a, (const uint32_t*)h->sh->d_g2l, in, n);
    return hip_check(h, hipGetLastError(), "k_frontier_import");
}

// The delivery kernel changed (gsim_set_kernel_variant): the fresh bits are
// kept only by the topic-major one.
void deliver_blocks_changed(gsim_handle* h)
{
    h->dl->tm_cn = -1;          // the next k_send_tm launch rebuilds its block table
}

int32_t* deliver_slot_last(gsim_handle* h) { return h->dl ? h->dl->d_slot_last : nullptr; }

// The seen-set layout (gsim_internal.h Cells) for the current slot masks:
// each slot's first cell, the member bitmaps of the topics only some peers
// hold (sub-rings only: a shared ring's slot may carry any topic), and the
// number of cells.
struct CellLayout {
    std::vector<uint64_t> cbase, mbits;
    std::vector<uint32_t> mpre;
    uint64_t sparse = 0;
    size_t cells = 0;
    // member-major gossip (sub-rings of at most kMmMaxSlots slots): members per
    // topic in peer order (sparse topics), offsets, counts
    std::vector<uint32_t> mlist;
    std::vector<int64_t> mloff, mcount;
};
constexpr int64_t kMmMaxSlots = kMaxRing / 8;   // k_gossip_count_mm's slot list

static CellLayout cell_layout(const gsim_handle* h, const gsim_msg_config& cfg)
{
    CellLayout L;
    const int64_t N = h->n, ring = cfg.ring, R = cfg.topic_slots;
    const int32_t T = std::max(1, h->t);
    const int64_t nw = (N + 63) / 64;
    L.cbase.assign((size_t)ring, 0);
    if (R <= 0) {
        for (int64_t m = 0; m < ring; ++m) L.cbase[(size_t)m] = (uint64_t)(m * N);
        L.cells = (size_t)(ring * N);
        return L;
    }
    std::vector<int64_t> M((size_t)T, N);
    if (!h->smask.empty()) {
        std::fill(M.begin(), M.end(), 0);
        for (int64_t p = 0; p < N; ++p)
            for (uint64_t b = h->smask[(size_t)p]; b; b &= b - 1) M[(size_t)__builtin_ctzll(b)]++;
        for (int32_t t = 0; t < T; ++t)
            if (M[(size_t)t] < N) L.sparse |= 1ull << t;
    }
    uint64_t off = 0;
    for (int32_t t = 0; t < T; ++t)
        for (int64_t k = 0; k < R; ++k) {
            L.cbase[(size_t)(t * R + k)] = off;
            off += (uint64_t)M[(size_t)t];
        }
    L.cells = (size_t)off;
    if (L.sparse) {
        L.mbits.assign((size_t)T * (size_t)nw, 0);
        L.mpre.assign((size_t)T * (size_t)nw, 0);
        for (int64_t p = 0; p < N; ++p)
            for (uint64_t b = h->smask[(size_t)p] & L.sparse; b; b &= b - 1)
                L.mbits[(size_t)__builtin_ctzll(b) * (size_t)nw + (size_t)(p >> 6)] |= 1ull << (p & 63);
        for (int32_t t = 0; t < T; ++t) {
            uint32_t acc = 0;
            for (int64_t w = 0; w < nw; ++w) {
                L.mpre[(size_t)t * (size_t)nw + (size_t)w] = acc;
                acc += (uint32_t)__builtin_popcountll(L.mbits[(size_t)t * (size_t)nw + (size_t)w]);
            }
        }
        if (R <= kMmMaxSlots) {
            L.mloff.assign((size_t)T, -1);
            L.mcount.assign(M.begin(), M.end());
            int64_t off = 0;
            for (int32_t t = 0; t < T; ++t)
                if ((L.sparse >> t) & 1ull) { L.mloff[(size_t)t] = off; off += M[(size_t)t]; }
            L.mlist.assign((size_t)off, 0);
            std::vector<int64_t> fill(L.mloff);
            for (int64_t p = 0; p < N; ++p)
                for (uint64_t b = h->smask[(size_t)p] & L.sparse; b; b &= b - 1)
                    L.mlist[(size_t)fill[(size_t)__builtin_ctzll(b)]++] = (uint32_t)p;
        }
    }
    return L;
}

// Install a layout: bases, member tables (cells allocated by the caller).
static hipError_t install_layout(gsim_handle* h, Deliver* d, const CellLayout& L)
{
    hipError_t e = hipSuccess;
    auto fr = [](void* p) { if (p) (void)hipFree(p); };
    fr(d->d_cbase); fr(d->d_mbits); fr(d->d_mpre);
    fr(d->d_mlist); fr(d->d_mloff); fr(d->d_mcount); fr(d->d_mmtab); fr(d->d_mctab); fr(d->d_ihm); fr(d->d_mmb);
    d->d_cbase = nullptr; d->d_mbits = nullptr; d->d_mpre = nullptr;
    d->d_mlist = nullptr; d->d_mloff = nullptr; d->d_mcount = nullptr; d->d_mmtab = nullptr; d->d_mctab = nullptr;
    d->d_ihm = nullptr; d->d_mmb = nullptr;
    e = hipMalloc((void**)&d->d_cbase, std::max<size_t>(L.cbase.size() * 8, 8));
    if (e == hipSuccess) e = stream_copy(h, d->d_cbase, L.cbase.data(), L.cbase.size() * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess && L.sparse) {
        e = hipMalloc((void**)&d->d_mbits, L.mbits.size() * 8);
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_mpre, L.mpre.size() * 4);
        if (e == hipSuccess) e = stream_copy(h, d->d_mbits, L.mbits.data(), L.mbits.size() * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = stream_copy(h, d->d_mpre, L.mpre.data(), L.mpre.size() * 4, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && !L.mloff.empty()) {
        const size_t T = L.mloff.size();
        d->mmtab.assign(T + 1, 0);
        d->mctab.assign(T + 1, 0);
        for (size_t t = 0; t < T; ++t) {
            d->mmtab[t + 1] = d->mmtab[t] + (uint32_t)((L.mcount[t] + 255) / 256);
            d->mctab[t + 1] = d->mctab[t] + (uint32_t)((L.mcount[t] + 1023) / 1024);
        }
        e = hipMalloc((void**)&d->d_mlist, std::max<size_t>(L.mlist.size() * 4, 4));
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_mloff, T * 8);
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_mcount, T * 8);
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_mmtab, (T + 1) * 4);
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_mctab, (T + 1) * 4);
        if (e == hipSuccess && !L.mlist.empty())
            e = stream_copy(h, d->d_mlist, L.mlist.data(), L.mlist.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = stream_copy(h, d->d_mloff, L.mloff.data(), T * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = stream_copy(h, d->d_mcount, L.mcount.data(), T * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = stream_copy(h, d->d_mmtab, d->mmtab.data(), (T + 1) * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = stream_copy(h, d->d_mctab, d->mctab.data(), (T + 1) * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess && GSIM_IH_MASK && d->cfg.topic_slots > 0 && d->cfg.topic_slots <= kIhMaskSlots) {
            std::vector<int64_t> mmb(T, 0);
            int64_t tot = 0;
            for (size_t t = 0; t < T; ++t) { mmb[t] = tot; tot += L.mcount[t]; }
            e = hipMalloc((void**)&d->d_ihm, std::max<size_t>((size_t)tot * 32, 32));
            if (e == hipSuccess) e = hipMalloc((void**)&d->d_mmb, T * 8);
            if (e == hipSuccess) e = stream_copy(h, d->d_mmb, mmb.data(), T * 8, hipMemcpyHostToDevice);
        }
    }
    d->cbase = L.cbase;
    d->sparse = L.sparse;
    d->cell_nw = (h->n + 63) / 64;
    d->n_peers = h->n;
    d->n_cells = L.cells;
    return e;
}

// Copy every cell of the old layout that the new one keeps (members of both),
// the new members' cells unseen.
__global__ void k_cell_relayout(Cells o, Cells n, const uint32_t* mtopic, int64_t ring, int64_t N)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < ring * N; x += stride) {
        const uint32_t m = (uint32_t)(x / N), p = (uint32_t)(x - (int64_t)m * N);
        const int32_t t = (int32_t)mtopic[m];
        const int64_t ni = n.idx(m, t, p);
        if (ni >= 0) n.cell[ni] = o.get(m, t, p);
    }
}

uint8_t** deliver_gsel_slot(gsim_handle* h)
{
    static uint8_t* none = nullptr;
    return h->dl ? &h->dl->d_gsel : &none;
}

// The topic slot masks grew (ensure_slots): the arrays were re-laid out; the
// delivery's mesh masks are rebuilt from the moved router flags, and the
// seen-set's member spaces follow the masks (new members get unseen cells).
int slots_changed(gsim_handle* h)
{
    Deliver* d = h->dl;
    if (!d) return GSIM_OK;
    d->mask_version = 0;
    if (d->cfg.topic_slots <= 0) return GSIM_OK;
    CellLayout L = cell_layout(h, d->cfg);
    if (L.cells == d->n_cells && L.sparse == d->sparse && L.mbits.empty() == (d->d_mbits == nullptr)) {
        // same sizes: unchanged memberships keep every cell (a member set can
        // only grow, so equal counts mean equal sets)
        return GSIM_OK;
    }
    const Cells old = deliver_cells(d);
    uint64_t* old_cbase = d->d_cbase;
    uint64_t* old_mbits = d->d_mbits;
    uint32_t* old_mpre = d->d_mpre;
    uint64_t* cell1 = nullptr;
    hipError_t e = hipMalloc((void**)&cell1, std::max<size_t>(L.cells * 8, 8));
    if (e != hipSuccess) return hip_check(h, e, "seen-set re-layout");
    d->d_cbase = nullptr; d->d_mbits = nullptr; d->d_mpre = nullptr;   // kept in `old` until copied
    e = install_layout(h, d, L);
    if (e == hipSuccess) {
        d->d_cell = cell1;
        const Cells nw = deliver_cells(d);
        const int64_t n = (int64_t)d->cfg.ring * h->n;
        hipLaunchKernelGGL(k_cell_relayout, dim3((uint32_t)std::min<int64_t>((n + 255) / 256, 65536)), dim3(256), 0,
                           h->stream, old, nw, (const uint32_t*)d->d_mtopic, (int64_t)d->cfg.ring, h->n);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    }
    (void)hipFree(old.cell);
    if (old_cbase) (void)hipFree(old_cbase);
    if (old_mbits) (void)hipFree(old_mbits);
    if (old_mpre) (void)hipFree(old_mpre);
    return hip_check(h, e, "k_cell_relayout");
}

extern "C" {

int gsim_msgs_init(gsim_handle* h, const gsim_msg_config* cfg)
{
    if (!h || !cfg) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->e == 0) { h->err = "no graph loaded"; return GSIM_ESTATE; }
    if (cfg->ring <= 0 || cfg->ring > kMaxRing || cfg->rounds < 2 || cfg->heartbeat_ns <= 0) {
        h->err = "invalid message configuration (ring must be in [1, 8192], rounds >= 2, heartbeat > 0)";
        return GSIM_EINVAL;
    }
    if (h->e >= (int64_t)kEdgeMask || h->n >= (int64_t)kPeerMask) {
        h->err = "too many edges or peers for the seen-set claim encoding (< 2^30 - 1)";
        return GSIM_ERANGE;
    }
    if (cfg->topic_slots < 0 || (cfg->topic_slots > 0 && (int64_t)cfg->ring != cfg->topic_slots * std::max(1, h->t))) {
        h->err = "topic_slots: every topic owns topic_slots ring slots, so ring must be n_topics * topic_slots";
        return GSIM_EINVAL;
    }
    (void)hipStreamSynchronize(h->stream);
    free_deliver(h);
    Deliver* d = new Deliver();
    d->cfg = *cfg;
    const CellLayout layout = cell_layout(h, *cfg);
    d->tcount.assign((size_t)std::max(1, h->t), 0);
    d->pubw.assign((size_t)kPubTicks * (size_t)std::max(1, h->t), 0);
    d->pubw_tick.assign((size_t)kPubTicks, -1);
    d->pub_bound = 0;
    d->applied_tick = 0;
    const size_t ring = (size_t)cfg->ring, N = (size_t)h->n, T = (size_t)std::max(1, h->t);
    const size_t CN = N;   // every local peer has cells (a shard's ghost cells: imported first-seen rounds)
    const size_t words = (size_t)nnew_words(d);
    hipError_t e = hipSuccess;
    auto A = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, std::max<size_t>(bytes, 4));
        if (e == hipSuccess) h->bytes_allocated += bytes;
    };
    A((void**)&d->d_mtopic, ring * 4);
    A((void**)&d->d_morigin, ring * 4);
    A((void**)&d->d_minv, ring);
    A((void**)&d->d_mlat, ring);
    A((void**)&d->d_mid, ring * 8);
    A((void**)&d->d_cell, layout.cells * 8);
    A((void**)&d->d_seenbm, ring * ((CN + 63) / 64) * 8);
    A((void**)&d->d_fresh, ring * ((CN + 63) / 64) * 8);
    A((void**)&d->d_fsum, ring * (((CN + 63) / 64 + 63) / 64) * 8);
    A((void**)&d->d_mmask, T * N * 8);
    A((void**)&d->d_tmtab, (2 * 64 + 1) * 4);
    d->tm_cn = -1;
    if (cfg->topic_slots > 0) {
        // claim list for member-compacted cells (list_commit): a round's first
        // deliveries, 4 N entries; more overflow into k_commit's word scan (and
        // the round's send into the fresh-bit scan).  c5 at 10M, ticks 2-5: 2 N
        // overflowed in the busy rounds, 346.7 ms per tick (send 75.1, commit
        // 63.7); 4 N 293.0 (50.7, 34.2); 8 N the same (gpurun_out/r05l)
#ifndef GSIM_CLIST_MULT
#define GSIM_CLIST_MULT 4
#endif
        // (gsim_msg_config.max_frontier > 0: that many claim-list entries and half
        // as many per forwarder list, a memory bound; overflow stays exact)
        d->clist_cap = cfg->max_frontier > 0 ? std::max<int64_t>(cfg->max_frontier / kClSub, 1)
                                             : std::max<int64_t>(GSIM_CLIST_MULT * (int64_t)N, 1 << 20) / kClSub;
        A((void**)&d->d_clist, (size_t)d->clist_cap * kClSub * 8);
        A((void**)&d->d_clist_n, (kClSub + 1) * kClStride * 4);
        if (e == hipSuccess) e = hipMemsetAsync(d->d_clist_n, 0, (kClSub + 1) * kClStride * 4, h->stream);
        // forwarder lists: a round's committed claims (the claim list's capacity:
        // more overflow into the scan) and its publications
        d->flist_cap = cfg->max_frontier > 0 ? std::max<int64_t>(cfg->max_frontier / 2, 64)
                                             : d->clist_cap * kClSub + (1 << 16);
        A((void**)&d->d_flist, (size_t)d->flist_cap * 2 * 8);
        A((void**)&d->d_fst, (kFstBad + kFstStride) * 4);
        if (e == hipSuccess) e = hipMemsetAsync(d->d_fst, 0, (kFstBad + kFstStride) * 4, h->stream);
        d->flist_round = -1;
    }
    if (h->max_degree > 64 && e == hipSuccess) {
        // hub rows and their mesh lists (k_hub_mesh)
        uint32_t* cnt = nullptr;
        uint32_t nh = 0;
        e = hipMalloc((void**)&cnt, 4);
        if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, 4, h->stream);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_hub_index, dim3(1024), dim3(256), 0, h->stream, (const uint32_t*)h->d_row_ptr, h->n,
                               (uint32_t*)nullptr, (uint32_t*)nullptr, cnt);
            e = hipMemcpyAsync(&nh, cnt, 4, hipMemcpyDeviceToHost, h->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        }
        const int64_t words = (int64_t)nh * (int64_t)T * (1 + kHubMesh);
        if (e == hipSuccess && nh && words < (int64_t)kHubList) {
            d->nhub = nh;
            A((void**)&d->d_hidx, N * 4);
            A((void**)&d->d_hrow, (size_t)nh * 4);
            A((void**)&d->d_hlist, (size_t)words * 4);
            if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, 4, h->stream);
            if (e == hipSuccess)
                hipLaunchKernelGGL(k_hub_index, dim3(1024), dim3(256), 0, h->stream, (const uint32_t*)h->d_row_ptr, h->n,
                                   d->d_hidx, d->d_hrow, cnt);
            if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        }
        if (cnt) (void)hipFree(cnt);
        d->hub_round = -1;
    }
    A((void**)&d->d_mpub, ring * 4);
    A((void**)&d->d_roff, (size_t)cfg->rounds * 8);
    A((void**)&d->d_lastput, T * N * 4);
    A((void**)&d->d_nnew, 2 * words * 4);
    A((void**)&d->d_stats, kStatLanes * kStatStride * 8);
    // promises live from round 0 of tick k until the first heartbeat after
    // round_time(kR) + IWantFollowupTime; one spare ring index
    {
        const int64_t hb = cfg->heartbeat_ns;
        const int64_t span = hb / (cfg->rounds + 1) + h->gp.iwant_followup_time_ns;
        d->prom_ticks = (int32_t)std::min<int64_t>(span / hb + 2, 64);
        d->prom_made.assign((size_t)d->prom_ticks, -1);
    }
    d->resp_cap = cfg->max_arrivals > 0 ? cfg->max_arrivals : std::max<int64_t>(8 * h->n, 1 << 20);
    A((void**)&d->d_slot_last, ring * 4);
    A((void**)&d->d_gsel, (size_t)std::max(1, h->S) * (size_t)h->e);
    A((void**)&d->d_gcount, 2 * ring * 4);
    A((void**)&d->d_gstate, (size_t)h->e);
    A((void**)&d->d_resp, (size_t)d->resp_cap * 8);
    A((void**)&d->d_nresp, 4 * 4);
    d->ptx_w = (int32_t)std::max<uint32_t>(h->max_degree, 1u);
    A((void**)&d->d_peertx, ring * (size_t)d->ptx_w);
    A((void**)&d->d_prom, (size_t)d->prom_ticks * (size_t)h->e * 4);
    A((void**)&d->d_pcand, (size_t)h->e * 8);
    A((void**)&d->d_behaviour, N);
    A((void**)&d->d_gstats, 4 * 8);
    if (e != hipSuccess) {
        dl_free(d);
        h->err = std::string("message ring allocation: ") + hipGetErrorString(e);
        return e == hipErrorOutOfMemory ? GSIM_ENOMEM : GSIM_EDEVICE;
    }
    h->dl = d;
    e = install_layout(h, d, layout);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_cell, 0xFF, layout.cells * 8, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_seenbm, 0, ring * ((CN + 63) / 64) * 8, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_fresh, 0, ring * ((CN + 63) / 64) * 8, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_fsum, 0, ring * (((CN + 63) / 64 + 63) / 64) * 8, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_mpub, 0, ring * 4, h->stream);
    if (e == hipSuccess) {
        std::vector<int64_t> roff((size_t)cfg->rounds);
        for (int32_t r = 0; r < cfg->rounds; ++r)
            roff[(size_t)r] = (int64_t)(r + 1) * cfg->heartbeat_ns / (cfg->rounds + 1);
        e = stream_copy(h, d->d_roff, roff.data(), roff.size() * 8, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipMemsetAsync(d->d_lastput, 0xFF, T * N * 4, h->stream);
    if (e == hipSuccess) {
        // a sub-ring slot carries its topic from the start (the cells' member space)
        std::vector<uint32_t> mt(ring, 0);
        if (cfg->topic_slots > 0)
            for (size_t m = 0; m < ring; ++m) mt[m] = (uint32_t)(m / (size_t)cfg->topic_slots);
        e = stream_copy(h, d->d_mtopic, mt.data(), ring * 4, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipMemsetAsync(d->d_morigin, 0, ring * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_minv, 0, ring, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_mlat, 0, ring, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_nnew, 0, 2 * words * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_stats, 0, kStatLanes * kStatStride * 8, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_slot_last, 0xFF, ring * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_gsel, 0, (size_t)std::max(1, h->S) * (size_t)h->e, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_gstate, 0, (size_t)h->e, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_nresp, 0, 4 * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_peertx, 0, ring * (size_t)d->ptx_w, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_prom, 0xFF, (size_t)d->prom_ticks * (size_t)h->e * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_pcand, 0xFF, (size_t)h->e * 8, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_behaviour, 0, N, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_gstats, 0, 4 * 8, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return hip_check(h, e, "gsim_msgs_init");
}

}  // extern "C"

// The ring slot of each message of a publish batch: its topic's next slot of
// a sub-ring (tcount: the topic's publications so far, advanced here), else
// id % ring.
static void batch_slots(const Deliver* d, std::vector<int64_t>& tcount, const gsim_msg* msgs, int32_t count,
                        uint32_t* slots)
{
    for (int32_t m = 0; m < count; ++m) {
        if (d->cfg.topic_slots > 0) {
            const int64_t R = d->cfg.topic_slots, t = msgs[m].topic;
            if ((size_t)t >= tcount.size()) { slots[m] = 0; continue; }   // (refused by the caller's checks)
            int64_t k = tcount[(size_t)t];
            for (int32_t q = 0; q < m; ++q) k += msgs[q].topic == msgs[m].topic;
            slots[m] = (uint32_t)(t * R + k % R);
        } else {
            slots[m] = (uint32_t)(msgs[m].id % (uint64_t)d->cfg.ring);
        }
    }
    for (int32_t m = 0; m < count && d->cfg.topic_slots > 0; ++m)
        if ((size_t)msgs[m].topic < tcount.size()) tcount[msgs[m].topic]++;
}

// gsim_publish; d_src / d_slots: the batch already on the device (gsim_step's
// schedule) -- no upload
static int publish_impl(gsim_handle* h, const gsim_msg* msgs, int32_t count, int64_t round, const gsim_msg* d_src,
                        const uint32_t* d_slots)
{
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    if (count < 0 || (count > 0 && !msgs) || round < 0) return GSIM_EINVAL;
    if (count == 0) return GSIM_OK;
    if (d->next_round >= 0 && round != d->next_round) {
        h->err = "messages must be published for the next round";
        return GSIM_ESTATE;
    }
    std::vector<uint32_t> slots((size_t)count);
    {
        std::vector<int64_t> tc(d->tcount);         // (advanced below, once the batch is accepted)
        batch_slots(d, tc, msgs, count, slots.data());
    }
    for (int32_t m = 0; m < count; ++m) {
        // a shard gets every message; an origin that is not one of its peers is 0xFFFFFFFF
        const bool foreign = h->sh && msgs[m].origin == 0xFFFFFFFFu;
        if (msgs[m].topic >= (uint32_t)std::max(1, h->t) || ((int64_t)msgs[m].origin >= h->n && !foreign) ||
            msgs[m].verdict > GSIM_VERDICT_SIGNATURE) {
            h->err = "message topic or origin out of range";
            return GSIM_EINVAL;
        }
        if (msgs[m].vdelay > GSIM_MAX_VDELAY) { h->err = "vdelay above GSIM_MAX_VDELAY"; return GSIM_EINVAL; }
        if (msgs[m].vdelay && h->gt) {
            h->err = "a validation latency (vdelay) cannot be combined with the peer gater";
            return GSIM_ESTATE;
        }
        if (msgs[m].vdelay && h->sh && !h->sh->push) {
            h->err = "a validation latency (vdelay) on shards needs the copy push (GSIM_SHARD_PULL unset)";
            return GSIM_ERANGE;
        }
    }
    std::vector<uint32_t> sorted(slots);
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end()) {
        h->err = "two messages of one publish batch share a ring slot";
        return GSIM_EINVAL;
    }
    if (!h->smask.empty()) {
        // an origin outside its topic publishes to its fanout: that state
        // lives in its topic slots
        std::vector<uint64_t> need;
        for (int32_t m = 0; m < count; ++m) {
            const uint32_t o = msgs[m].origin;
            if ((int64_t)o >= h->n || ((h->smask[o] >> msgs[m].topic) & 1ull)) continue;
            if (need.empty()) need.assign((size_t)h->n, 0);
            need[o] |= 1ull << msgs[m].topic;
        }
        if (!need.empty()) {
            const int rc = ensure_slots(h, need.data());
            if (rc) return rc;
        }
    }
    hipError_t e = hipSuccess;
    if (!d_src && count > d->pub_cap) {
        (void)hipStreamSynchronize(h->stream);
        if (d->d_pub) { (void)hipFree(d->d_pub); d->d_pub = nullptr; }
        if (d->d_pslot) { (void)hipFree(d->d_pslot); d->d_pslot = nullptr; }
        const int32_t cap = std::max(count, 256);
        e = hipMalloc((void**)&d->d_pub, sizeof(gsim_msg) * (size_t)cap);
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_pslot, sizeof(uint32_t) * (size_t)cap);
        if (e != hipSuccess) { d->pub_cap = 0; return hip_check(h, e, "hipMalloc publish"); }
        d->pub_cap = cap;
    }
    if (!d->lat_on && std::any_of(msgs, msgs + count, [](const gsim_msg& x) { return x.vdelay != 0; })) {
        // first message with a validation latency: the pending-copy queues
        // (each plane holds the copies of at most GSIM_MAX_VDELAY rounds;
        // gsim_msg_config.max_arrivals raises it)
        const int w = nnew_words(d);
        // dense layout (every peer holds every topic's records, no slot relayout):
        // the copies k_send_tm makes pending are counted per record, the queue
        // keeps the winners' P2, the IWANT responses and counts that overflow
        const bool counts = h->smask.empty() && !h->sh;
        const size_t vpe = ((size_t)std::max(1, h->t) * (size_t)h->e + 7) & ~(size_t)7;
        d->vq_cap = counts ? std::max<int64_t>(std::max<int64_t>(4 * h->n, 1 << 16), d->cfg.max_arrivals)
                           : std::max<int64_t>(std::max<int64_t>(4 * h->e, 1 << 16), d->cfg.max_arrivals);
        d->vq_cap = (d->vq_cap / kVqSub + 1) * kVqSub * 2;     // sub-lists of twice the average share
        e = hipMalloc((void**)&d->d_vq, sizeof(uint64_t) * (size_t)kVqPlanes * (size_t)d->vq_cap);
        if (e == hipSuccess && counts) e = hipMalloc((void**)&d->d_vpc, 2 * (size_t)kVqPlanes * vpe);
        if (e == hipSuccess && counts) e = hipMemsetAsync(d->d_vpc, 0, 2 * (size_t)kVqPlanes * vpe, h->stream);
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_vqn, sizeof(uint32_t) * (size_t)kVqnWords);
        if (e == hipSuccess) e = hipMalloc((void**)&d->d_hist, sizeof(uint32_t) * (size_t)kVqPlanes * (size_t)w);
        if (e == hipSuccess) e = hipMemsetAsync(d->d_vqn, 0, sizeof(uint32_t) * (size_t)kVqnWords, h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(d->d_hist, 0, sizeof(uint32_t) * (size_t)kVqPlanes * (size_t)w, h->stream);
        if (e != hipSuccess) return hip_check(h, e, "validation queues");
        d->lat_on = true;
    }
    {
        // the last round's claims are committed before slots are reset (k_reset_slots)
        const int rcf = deliver_flush(h);
        if (rcf) return rcf;
    }
    if (!d_src) {
        e = hipMemcpyAsync(d->d_pub, msgs, sizeof(gsim_msg) * (size_t)count, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(d->d_pslot, slots.data(), sizeof(uint32_t) * (size_t)count, hipMemcpyHostToDevice,
                               h->stream);
        if (e != hipSuccess) return hip_check(h, e, "publish upload");
        d_src = d->d_pub;
        d_slots = d->d_pslot;
    }
    {
        std::vector<int64_t>& tc = d->tcount;
        batch_slots(d, tc, msgs, count, slots.data());   // (advances the topics' counts)
    }
    {
        // the publication window (RoundArgs::mcnt_fast)
        const int64_t tick = round / std::max(1, d->cfg.rounds);
        const size_t T = (size_t)std::max(1, h->t), row = (size_t)(tick % kPubTicks);
        if (d->pubw_tick[row] != tick) {
            std::fill(d->pubw.begin() + (int64_t)(row * T), d->pubw.begin() + (int64_t)((row + 1) * T), 0);
            d->pubw_tick[row] = tick;
        }
        for (int32_t m = 0; m < count; ++m) d->pubw[row * T + msgs[m].topic]++;
        // a copy of a message comes at most HistoryLength + 2 ticks after its
        // publication (forwarded, or an IWANT answer from an mcache): the
        // pending increments since the last application are copies of messages
        // published after applied_tick - W
        const int64_t W = (int64_t)h->gp.history_length + 3;
        const int64_t from = std::min(tick, d->applied_tick) - W;
        int32_t mx = 0;
        if (tick - from > kPubTicks) {
            mx = INT32_MAX;                                  // beyond the window's memory: no bound
        } else {
            for (size_t t = 0; t < T; ++t) {
                int32_t sum = 0;
                for (size_t r = 0; r < (size_t)kPubTicks; ++r)
                    if (d->pubw_tick[r] > from) sum += d->pubw[r * T + t];
                mx = std::max(mx, sum);
            }
        }
        d->pub_bound = mx;
    }
    ProfScope ps(h, GSIM_K_PUBLISH);
    RoundArgs a = make_round_args(h, round);
    const int64_t per_block = 256 * 16;
    const int gx = (int)std::min<int64_t>((h->n + per_block - 1) / per_block, 1024);
    hipLaunchKernelGGL(k_reset_slots, dim3(std::max(gx, 1), count), dim3(256), 0, h->stream, a, d_slots, count);
    hipLaunchKernelGGL(k_publish, dim3((count + 255) / 256), dim3(256), 0, h->stream, a, d_src, d_slots, count);
    d->next_round = round;
    int rc = hip_check(h, hipGetLastError(), "k_publish");
    // origins that have not joined the topic publish to their fanout
    if (!rc) rc = launch_fanout_publish(h, d_src, count, round, round_time_host(d, round));
    return rc;
}

extern "C" {

int gsim_publish(gsim_handle* h, const gsim_msg* msgs, int32_t count, int64_t round)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    return publish_impl(h, msgs, count, round, nullptr, nullptr);
}

#ifdef GSIM_DIAG_IH
// the IHAVE walk's diagnostic counters (not part of gsim.h): read, then reset
extern "C" int gsim_diag_ih_counts(gsim_handle* h, uint64_t* out16)
{
    if (!h || !out16) return GSIM_EINVAL;
    if (hipStreamSynchronize(h->stream) != hipSuccess) return GSIM_EDEVICE;
    unsigned long long z[16] = {};
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_ih_diag), sizeof(z)) != hipSuccess) return GSIM_EDEVICE;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ih_diag), z, sizeof(z)) != hipSuccess) return GSIM_EDEVICE;
    return GSIM_OK;
}
#endif

int gsim_round(gsim_handle* h, int64_t round)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->sh) { h->err = "a shard's rounds run through its group (gsim_group_round)"; return GSIM_ESTATE; }
    int rc = deliver_round_prepare(h, round);
    if (!rc) rc = deliver_round_send(h, round);
    if (!rc) rc = deliver_round_post(h, round);
    if (!rc) rc = deliver_round_control(h, round);
    if (!rc) rc = deliver_round_ihave(h, round);
    if (!rc) rc = deliver_round_validate(h, round);
    if (rc) return rc;
    deliver_round_end(h, round);
    return GSIM_OK;
}

int gsim_step(gsim_handle* h, uint64_t tick, int32_t n_ticks, const gsim_msg* msgs, const int64_t* round_off)
{
    if (!h || n_ticks < 0) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->sh) { h->err = "a shard's ticks run through its group"; return GSIM_ESTATE; }
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    if (n_ticks == 0) return GSIM_OK;
    const int R = d->cfg.rounds;
    const int64_t nr = (int64_t)n_ticks * R;
    if ((msgs == nullptr) != (round_off == nullptr)) return GSIM_EINVAL;
    int64_t nmsg = 0;
    if (round_off) {
        if (round_off[0] != 0) return GSIM_EINVAL;
        for (int64_t q = 0; q < nr; ++q)
            if (round_off[q + 1] < round_off[q] || round_off[q + 1] - round_off[q] > INT32_MAX) return GSIM_EINVAL;
        nmsg = round_off[nr];
    }
    int rc = deliver_check_errors(h);                // what the last call left
    if (rc) return rc;
    if (nmsg > 0) {
        // the schedule's ring slots as the publications will take them (the
        // topics' sub-ring counts advance batch by batch), then one upload
        std::vector<uint32_t> slots((size_t)nmsg);
        std::vector<int64_t> tc(d->tcount);
        for (int64_t q = 0; q < nr; ++q)
            batch_slots(d, tc, msgs + round_off[q], (int32_t)(round_off[q + 1] - round_off[q]),
                        slots.data() + round_off[q]);
        hipError_t e = hipSuccess;
        if (nmsg > d->sched_cap) {
            e = hipStreamSynchronize(h->stream);
            if (d->d_sched) { (void)hipFree(d->d_sched); d->d_sched = nullptr; }
            if (d->d_sslot) { (void)hipFree(d->d_sslot); d->d_sslot = nullptr; }
            d->sched_cap = 0;
            const int64_t cap = std::max<int64_t>(nmsg, 4096);
            if (e == hipSuccess) e = hipMalloc((void**)&d->d_sched, sizeof(gsim_msg) * (size_t)cap);
            if (e == hipSuccess) e = hipMalloc((void**)&d->d_sslot, sizeof(uint32_t) * (size_t)cap);
            if (e != hipSuccess) return hip_check(h, e, "gsim_step schedule");
            d->sched_cap = cap;
        }
        // (no kernel reads the buffers any more: every call ends synchronised)
        if (e == hipSuccess)
            e = hipMemcpyAsync(d->d_sched, msgs, sizeof(gsim_msg) * (size_t)nmsg, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(d->d_sslot, slots.data(), sizeof(uint32_t) * (size_t)nmsg, hipMemcpyHostToDevice,
                               h->stream);
        if (e != hipSuccess) return hip_check(h, e, "gsim_step schedule upload");
    }
    h->in_step = true;
    for (int32_t k = 0; k < n_ticks && !rc; ++k) {
        const uint64_t tk = tick + (uint64_t)k;
        const int64_t now = d->cfg.t0_ns + (int64_t)tk * d->cfg.heartbeat_ns;
        rc = gsim_refresh_scores(h, now);
        if (!rc) rc = gsim_heartbeat(h, tk, now);
        for (int r = 0; r < R && !rc; ++r) {
            const int64_t q = (int64_t)k * R + r, g = (int64_t)tk * R + r;
            const int64_t o0 = round_off ? round_off[q] : 0, cnt = round_off ? round_off[q + 1] - o0 : 0;
            if (cnt > 0) rc = publish_impl(h, msgs + o0, (int32_t)cnt, g, d->d_sched + o0, d->d_sslot + o0);
            if (!rc) rc = gsim_round(h, g);
        }
    }
    h->in_step = false;
    if (!rc) rc = deliver_check_errors(h);         // one synchronisation per call
    return rc;
}

int gsim_msg_stats(gsim_handle* h, int64_t* out4)
{
    if (!h || !out4) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    unsigned long long sl[kStatLanes * kStatStride];
    uint32_t err[4] = {0, 0, 0, 0};
    hipError_t e = hipMemcpyAsync(sl, d->d_stats, sizeof(sl), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(err, d->d_nresp, sizeof(err), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_msg_stats");
    for (int k = 0; k < 4; ++k) {
        unsigned long long v = 0;
        for (int l = 0; l < kStatLanes; ++l) v += sl[l * kStatStride + k];
        out4[k] = (int64_t)v;
    }
    if (err[1]) { h->err = "IWANT responses overflowed their queue (raise gsim_msg_config.max_arrivals)"; return GSIM_ERANGE; }
    if (int rc = vq_check(h)) return rc;
    if (err[2]) {
        h->err = "a ring slot was republished while its message could still be gossiped or promised (raise ring)";
        return GSIM_ESTATE;
    }
    return GSIM_OK;
}

int gsim_gossip_stats(gsim_handle* h, int64_t* out4)
{
    if (!h || !out4) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    unsigned long long s[4];
    hipError_t e = hipMemcpyAsync(s, d->d_gstats, sizeof(s), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_gossip_stats");
    for (int k = 0; k < 4; ++k) out4[k] = (int64_t)s[k];
    return GSIM_OK;
}

int gsim_set_peer_behaviour(gsim_handle* h, const uint8_t* flags)
{
    if (!h || !flags) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    hipError_t e = hipMemcpyAsync(d->d_behaviour, flags, (size_t)h->n, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return hip_check(h, e, "gsim_set_peer_behaviour");
}

}  // extern "C"

// Diagnostic build only (GSIM_DIAG_PHASE): k_send_tm's phase clocks since the
// last call (all zero in a normal build), then reset.
extern "C" int gsim_diag_send_phases(gsim_handle* h, uint64_t* out8)
{
    if (!h || !out8) return GSIM_EINVAL;
    for (int k = 0; k < 8; ++k) out8[k] = 0;
#ifdef GSIM_DIAG_PHASE
    if (hipStreamSynchronize(h->stream) != hipSuccess) return GSIM_EDEVICE;
    unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_tm_diag), sizeof(v)) != hipSuccess) return GSIM_EDEVICE;
    for (int k = 0; k < 8; ++k) out8[k] = v[k];
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_tm_diag), z, sizeof(z)) != hipSuccess) return GSIM_EDEVICE;
#endif
    return GSIM_OK;
}
