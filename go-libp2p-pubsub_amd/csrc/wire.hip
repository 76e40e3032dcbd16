// The heartbeat's RPCs on the wire, encoded on the device
// (include/gsim_wire.h gsim_wire_heartbeat).
//
// At heartbeat k a router p sends each neighbour q at most one RPC: the
// GRAFTs and PRUNEs of sendGraftPrune (gossipsub.go:1672-1709) carrying, by
// piggybackGossip (1799-1807), the IHAVEs emitGossip queued for q
// (1711-1775), or those IHAVEs alone from flush (1777-1791).  The engine
// holds all of it right after its heartbeat: GRAFT / PRUNE bits in the
// parity-0 control inbox at the receiver's edge, emitGossip's targets in
// gsel at the sender's edge, and every router's mcache window in the seen
// cells (the first-seen round of each message it holds).
//
// Four passes over the senders [p0, p1):
//   k_wire_ids_count  per (p, t) with an IHAVE target: the ids of
//                     GetGossipIDs(t) (mcache.go:82-92) — messages of t whose
//                     first sight at p lies in the last HistoryGossip ticks,
//                     accepted or published by p;
//   k_wire_size       per edge: the RPC's encoded size (0: nothing sent);
//   (exclusive scans of both: id offsets, byte offsets, RPC indices)
//   k_wire_ids        per (p, t): the id list in GetGossipIDs order (newest
//                     history window first, each window in Put order: by
//                     round, the router's own publications first, then
//                     receipts by slot — the order the receiver handles a
//                     round's copies in);
//   k_wire_write      per edge: the bytes (rpc.pb.go field order).
// Integer/byte work bound by HBM (one pass over the senders' rows and flag
// planes, the window cells of the IHAVE senders, and the output bytes).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "gsim_internal.h"
#include "gsim_wire.h"
#include "philox.h"

namespace gsim {
namespace {

struct WireArgs {
    const uint32_t *row_ptr, *col, *rev, *owner;
    const uint8_t* ctl;           // parity-0 inbox [T][E] (receivers' edges)
    const uint8_t* gsel;          // [T][E] (senders' edges)
    const uint64_t* smask;        // topic slots of both arrays (gsim_internal.h; nullptr: dense)
    Cells cells;                  // the seen-set (gsim_internal.h)
    int64_t N, E;
    int32_t T, R;
    const uint32_t *mtopic, *morigin;
    const uint8_t* minv;
    const uint64_t* mid;
    const uint16_t* cand;         // candidate slots of each topic
    const int32_t* cand_ptr;      // [T + 1]
    int64_t g;                    // the tick's first round
    int64_t lo_round;             // first round of the gossip window
    uint32_t p0, p1;
    int64_t e0, e1;               // the senders' edges
    const uint8_t* names;         // topic names, concatenated
    const uint32_t* name_off;     // [T + 1]
    const uint8_t* peer_ids;      // [N][pid_len] or nullptr
    uint32_t pid_len;
    uint64_t backoff;
    uint64_t* n_pt;               // [(p1 - p0) * T + 1]
    uint64_t* id_off;             // [(p1 - p0) * T + 1]
    uint32_t* ids;                // slots, GetGossipIDs order
    uint64_t* rsize;              // [edges + 1]
    uint32_t* rflag;              // [edges + 1]
    uint64_t* roff;               // [edges + 1]
    uint32_t* rcnt;               // [edges + 1]
    uint8_t* out;
    gsim_wire_ref* refs;
    int32_t max_ihave;            // MaxIHaveLength
    uint32_t* err;                // [0] bit 0: an IHAVE target without ids; bit 1: a window longer than
                                  // MaxIHaveLength
    // makePrune's PX lists (gossipsub.go:1866-1906): a heartbeat PRUNE's is recomputed from the
    // live scores its k_px_emit read (pxs) and the same Philox keys; a Leave PRUNE's
    // (GSIM_CTL_UNSUB) was kept at the Leave (pxl entries of this tick)
    const uint8_t* rstate;
    const uint64_t* sub;
    const double* pxs;
    uint64_t seed;
    int64_t tick;
    int32_t prune_peers;
    const uint64_t* pxl;
    const uint32_t* pxl_tick;
    uint32_t n_pxl;
    uint64_t unsub_backoff;       // UnsubscribeBackoff / 1s: a Leave PRUNE's Backoff
};

constexpr int kWirePxMax = 64;    // PrunePeers the encoder lists (more: refused)

__device__ __forceinline__ uint32_t vlen(uint64_t v)
{
    uint32_t n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
}
__device__ __forceinline__ uint64_t ld(uint64_t n) { return 1 + vlen(n) + n; }

// first-seen round of a cell with the tick's rounds not begun: a pending
// claim is from round g - 1
__device__ __forceinline__ int64_t seen_round(uint64_t c, int64_t g)
{
    if (c == kUnseen64) return -1;
    const uint32_t hi = (uint32_t)(c >> 32);
    if (!(hi & kClaim)) return hi;
    return (((hi >> 30) & 1u) == (uint32_t)(g & 1)) ? g : g - 1;
}

// p put slot m in its mcache within the gossip window (mcache.Put of an
// accepted first delivery, or of its own publication); its round, else -1
__device__ __forceinline__ int64_t window_put(const WireArgs& a, uint32_t m, uint32_t p)
{
    const int64_t fr = seen_round(a.cells.get(m, (int32_t)a.mtopic[m], p), a.g);
    if (fr < a.lo_round || fr >= a.g) return -1;
    if (a.minv[m] != GSIM_VERDICT_ACCEPT && a.morigin[m] != p) return -1;
    return fr;
}

// the slot-layout entries (gsim_internal.h): gsel of edge e in its sender
// p's row, the inbox entry re in the receiver q's row
__device__ __forceinline__ bool gsel_at(const WireArgs& a, int32_t t, int64_t e, uint64_t mp)
{
    return a.gsel && slot_has(mp, t) && a.gsel[slot_idx(mp, t, a.E, e)] != 0;
}
__device__ __forceinline__ uint8_t ctl_at(const WireArgs& a, int32_t t, int64_t re, uint64_t mq)
{
    return slot_has(mq, t) ? a.ctl[slot_idx(mq, t, a.E, re)] : 0;
}

__global__ void k_wire_ids_count(WireArgs a)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = (int64_t)(a.p1 - a.p0) * a.T;
    if (k >= n) return;
    const uint32_t p = a.p0 + (uint32_t)(k / a.T);
    const int32_t t = (int32_t)(k % a.T);
    uint64_t cnt = 0;
    bool any = false;
    const uint64_t mp = smask_of(a.smask, p);
    for (uint32_t e = a.row_ptr[p]; e < a.row_ptr[p + 1] && !any; ++e) any = gsel_at(a, t, e, mp);
    if (any) {
        for (int32_t q = a.cand_ptr[t]; q < a.cand_ptr[t + 1]; ++q) cnt += window_put(a, a.cand[q], p) >= 0;
        if (!cnt) atomicOr(&a.err[0], 1u);                   // emitGossip has nothing to send
        // emitGossip would send each target its own random MaxIHaveLength-subset
        // (gossipsub.go:1763-1772), which is not encoded here
        if (cnt > (uint64_t)a.max_ihave) atomicOr(&a.err[0], 2u);
    }
    a.n_pt[k] = cnt;
}

// bytes of topic t's name as an optional string field
__device__ __forceinline__ uint64_t name_field(const WireArgs& a, int32_t t)
{
    return ld(a.name_off[t + 1] - a.name_off[t]);
}

__device__ __forceinline__ uint64_t ihave_body(const WireArgs& a, int32_t t, uint32_t n)
{
    return name_field(a, t) + (uint64_t)n * ld(a.pid_len + 8);
}

// The PX list of the PRUNE p -> col[e] in topic t (ctl: its inbox bits), in
// list order; returns its length.
__device__ uint32_t px_list(const WireArgs& a, int64_t e, uint32_t p, int32_t t, uint8_t ctl, uint32_t* out)
{
    if (!(ctl & GSIM_CTL_PX)) return 0;
    uint32_t n = 0;
    if (ctl & GSIM_CTL_UNSUB) {                              // Leave's: kept at the Leave
        for (uint32_t q = 0; q < a.n_pxl && n < kWirePxMax; ++q) {
            const uint64_t v = a.pxl[q];
            if ((uint32_t)v == (uint32_t)e && (int32_t)((v >> 32) & 63u) == t && a.pxl_tick[q] == (uint32_t)a.tick)
                out[n++] = (uint32_t)(v >> 38);
        }
        return n;
    }
    // the heartbeat's: getPeers(topic, PrunePeers, xp != p && Score(xp) >= 0) on the live
    // scores after the heartbeat, the PrunePeers smallest keys (k_px_emit)
    const uint32_t b = a.row_ptr[p], en = a.row_ptr[p + 1];
    uint64_t last = 0;
    for (int k = 0; k < a.prune_peers && k < kWirePxMax; ++k) {
        uint64_t best = ~0ull;
        uint32_t bx = 0xFFFFFFFFu;
        for (uint32_t q = b; q < en; ++q) {
            if ((int64_t)q == e) continue;
            const uint32_t x = a.col[q];
            if (!(a.rstate[q] & GSIM_ES_CONNECTED) || !((a.sub[x] >> t) & 1ull) || a.pxs[q] < 0.0) continue;
            const uint64_t key = px_key(px_base(a.seed, (uint32_t)a.tick, p, (uint32_t)t, P_PX, x), (uint32_t)(e - b), q - b);
            if ((k > 0 && key <= last) || key >= best) continue;
            best = key;
            bx = x;
        }
        if (bx == 0xFFFFFFFFu) break;
        last = best;
        out[n++] = bx;
    }
    return n;
}

__device__ __forceinline__ uint32_t pid_bytes(const WireArgs& a) { return a.pid_len ? a.pid_len : 4u; }

__device__ __forceinline__ uint64_t prune_body(const WireArgs& a, int32_t t, uint8_t ctl, uint32_t npx)
{
    const uint64_t bo = (ctl & GSIM_CTL_UNSUB) ? a.unsub_backoff : a.backoff;
    return name_field(a, t) + (uint64_t)npx * ld(ld(pid_bytes(a))) + 1 + vlen(bo);
}

// ControlMessage body of edge e (p -> col[e]); 0 and *any = false: no RPC
__device__ uint64_t control_body(const WireArgs& a, int64_t e, uint32_t p, bool* any)
{
    const int64_t re = a.rev[e];
    const int64_t base = (int64_t)(p - a.p0) * a.T;
    const uint64_t mp = smask_of(a.smask, p), mq = smask_of(a.smask, a.col[e]);
    uint64_t s = 0;
    bool x = false;
    for (int32_t t = 0; t < a.T; ++t) {
        const uint8_t c = ctl_at(a, t, re, mq);
        if (gsel_at(a, t, e, mp)) { s += ld(ihave_body(a, t, (uint32_t)a.n_pt[base + t])); x = true; }
        if (c & GSIM_CTL_GRAFT) { s += ld(name_field(a, t)); x = true; }
        if (c & GSIM_CTL_PRUNE) {
            uint32_t px[kWirePxMax];
            const uint32_t npx = px_list(a, e, p, t, c, px);
            s += ld(prune_body(a, t, c, npx));
            x = true;
        }
    }
    *any = x;
    return s;
}

__global__ void k_wire_size(WireArgs a)
{
    const int64_t e = a.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.e1) return;
    bool any = false;
    const uint64_t body = control_body(a, e, a.owner[e], &any);
    const uint64_t size = any ? ld(body) : 0;              // RPC.control = 3
    a.rsize[e - a.e0] = size;
    a.rflag[e - a.e0] = size ? 1u : 0u;
}

struct IdKey {
    int64_t window;   // ticks back from the newest window
    int64_t round;
    uint32_t own;     // 0: the router's publication
    uint64_t tie;     // own: message id; else slot
};

__device__ __forceinline__ bool key_less(const IdKey& x, const IdKey& y)
{
    if (x.window != y.window) return x.window < y.window;
    if (x.round != y.round) return x.round < y.round;
    if (x.own != y.own) return x.own < y.own;
    return x.tie < y.tie;
}

__device__ __forceinline__ IdKey id_key(const WireArgs& a, uint32_t m, uint32_t p)
{
    const int64_t fr = window_put(a, m, p);
    const bool own = a.morigin[m] == p;
    return IdKey{(a.g - 1) / a.R - fr / a.R, fr, own ? 0u : 1u, own ? a.mid[m] : (uint64_t)m};
}

__global__ void k_wire_ids(WireArgs a)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = (int64_t)(a.p1 - a.p0) * a.T;
    if (k >= n || !a.n_pt[k]) return;
    const uint32_t p = a.p0 + (uint32_t)(k / a.T);
    const int32_t t = (int32_t)(k % a.T);
    uint32_t* out = a.ids + a.id_off[k];
    uint32_t c = 0;
    for (int32_t q = a.cand_ptr[t]; q < a.cand_ptr[t + 1]; ++q) {
        const uint32_t m = a.cand[q];
        if (window_put(a, m, p) < 0) continue;
        // insertion into the sorted prefix (windows hold a handful of ids)
        const IdKey km = id_key(a, m, p);
        uint32_t j = c++;
        while (j > 0 && key_less(km, id_key(a, out[j - 1], p))) { out[j] = out[j - 1]; --j; }
        out[j] = m;
    }
}

struct ByteOut {
    uint8_t* p;
    __device__ void byte(uint8_t b) { *p++ = b; }
    __device__ void varint(uint64_t v)
    {
        while (v >= 0x80) { *p++ = (uint8_t)(v | 0x80); v >>= 7; }
        *p++ = (uint8_t)v;
    }
    __device__ void raw(const uint8_t* s, uint32_t n)
    {
        for (uint32_t q = 0; q < n; ++q) p[q] = s[q];
        p += n;
    }
};

__device__ void write_name(const WireArgs& a, ByteOut& w, uint8_t tag, int32_t t)
{
    const uint32_t b = a.name_off[t], n = a.name_off[t + 1] - b;
    w.byte(tag);
    w.varint(n);
    w.raw(a.names + b, n);
}

// message id: peer id of the origin (when given) || the gsim id, big-endian
__device__ void write_id(const WireArgs& a, ByteOut& w, uint32_t m)
{
    w.byte(0x12);                                          // ControlIHave.messageIDs = 2
    w.varint(a.pid_len + 8);
    if (a.pid_len) w.raw(a.peer_ids + (int64_t)a.morigin[m] * a.pid_len, a.pid_len);
    const uint64_t id = a.mid[m];
    for (int s = 56; s >= 0; s -= 8) w.byte((uint8_t)(id >> s));
}

__global__ void k_wire_write(WireArgs a)
{
    const int64_t e = a.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.e1 || !a.rsize[e - a.e0]) return;
    const uint32_t p = a.owner[e];
    bool any = false;
    const uint64_t body = control_body(a, e, p, &any);
    const int64_t re = a.rev[e];
    const int64_t base = (int64_t)(p - a.p0) * a.T;
    const uint64_t mp = smask_of(a.smask, p), mq = smask_of(a.smask, a.col[e]);
    ByteOut w{a.out + a.roff[e - a.e0]};
    w.byte(0x1a);                                          // RPC.control = 3
    w.varint(body);
    for (int32_t t = 0; t < a.T; ++t) {                    // ControlMessage.ihave = 1
        if (!gsel_at(a, t, e, mp)) continue;
        const uint32_t n = (uint32_t)a.n_pt[base + t];
        w.byte(0x0a);
        w.varint(ihave_body(a, t, n));
        write_name(a, w, 0x0a, t);                         // ControlIHave.topicID = 1
        const uint32_t* ids = a.ids + a.id_off[base + t];
        for (uint32_t q = 0; q < n; ++q) write_id(a, w, ids[q]);
    }
    for (int32_t t = 0; t < a.T; ++t) {                    // ControlMessage.graft = 3
        if (!(ctl_at(a, t, re, mq) & GSIM_CTL_GRAFT)) continue;
        w.byte(0x1a);
        w.varint(name_field(a, t));
        write_name(a, w, 0x0a, t);                         // ControlGraft.topicID = 1
    }
    for (int32_t t = 0; t < a.T; ++t) {                    // ControlMessage.prune = 4
        const uint8_t c = ctl_at(a, t, re, mq);
        if (!(c & GSIM_CTL_PRUNE)) continue;
        uint32_t px[kWirePxMax];
        const uint32_t npx = px_list(a, e, p, t, c, px);
        w.byte(0x22);
        w.varint(prune_body(a, t, c, npx));
        write_name(a, w, 0x0a, t);                         // ControlPrune.topicID = 1
        for (uint32_t q = 0; q < npx; ++q) {               // ControlPrune.peers = 2: PeerInfo{peerID = 1}
            const uint32_t L = pid_bytes(a);
            w.byte(0x12);
            w.varint(ld(L));
            w.byte(0x0a);
            w.varint(L);
            if (a.pid_len) {
                w.raw(a.peer_ids + (int64_t)px[q] * a.pid_len, a.pid_len);
            } else {
                for (int sh = 24; sh >= 0; sh -= 8) w.byte((uint8_t)(px[q] >> sh));
            }
        }
        w.byte(0x18);                                      // ControlPrune.backoff = 3
        w.varint((c & GSIM_CTL_UNSUB) ? a.unsub_backoff : a.backoff);
    }
    gsim_wire_ref r;
    r.from = p;
    r.to = a.col[e];
    r.len = (uint32_t)a.rsize[e - a.e0];
    r.pad = 0;
    r.offset = a.roff[e - a.e0];
    a.refs[a.rcnt[e - a.e0]] = r;
}

template <typename T>
int exclusive_scan(gsim_handle* h, const T* in, T* out, int64_t n, void** tmp, size_t* tmp_bytes)
{
    size_t need = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, (int)n, h->stream);
    if (e != hipSuccess) return hip_check(h, e, "wire scan size");
    if (need > *tmp_bytes) {
        if (*tmp) (void)hipFree(*tmp);
        *tmp = nullptr;
        e = hipMalloc(tmp, need);
        if (e != hipSuccess) { *tmp_bytes = 0; return hip_check(h, e, "wire scan scratch"); }
        *tmp_bytes = need;
    }
    e = hipcub::DeviceScan::ExclusiveSum(*tmp, need, in, out, (int)n, h->stream);
    return hip_check(h, e, "wire scan");
}

}  // namespace
}  // namespace gsim

using namespace gsim;

extern "C" int gsim_wire_heartbeat(gsim_handle* h, int64_t tick, uint32_t p0, uint32_t p1, const gsim_wire_names* names,
                                   uint8_t* d_out, uint64_t out_cap, gsim_wire_ref* d_refs, int64_t ref_cap,
                                   int64_t* n_rpcs, uint64_t* bytes)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->n == 0) { h->err = "no graph loaded (call gsim_load_graph first)"; return GSIM_ESTATE; }
    if (!names || !n_rpcs || !bytes || p0 > p1 || (int64_t)p1 > h->n) return GSIM_EINVAL;
    if (h->sh) { h->err = "gsim_wire_heartbeat runs on a single engine, not a shard"; return GSIM_ESTATE; }
    WireView v{};
    if (!deliver_wire_view(h, &v)) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    if (v.ihave_tick != tick) {
        h->err = "gsim_wire_heartbeat must follow gsim_heartbeat(tick) before the tick's first round";
        return GSIM_ESTATE;
    }
    const int32_t T = std::max(1, h->t);
    if (!names->topic_names) return GSIM_EINVAL;
    if (names->peer_id_len && !names->peer_ids) return GSIM_EINVAL;
    if (names->peer_id_len > 1024) return GSIM_ERANGE;

    // host tables: topic names and the candidate slots of each topic
    std::vector<uint32_t> name_off((size_t)T + 1, 0);
    std::vector<uint8_t> name_bytes;
    for (int32_t t = 0; t < T; ++t) {
        const gsim_bytes& b = names->topic_names[t];
        if (!b.p && b.n) return GSIM_EINVAL;
        name_bytes.insert(name_bytes.end(), b.p, b.p + b.n);
        name_off[(size_t)t + 1] = (uint32_t)name_bytes.size();
    }
    const int64_t g = tick * v.rounds;
    const int64_t lo_round = std::max<int64_t>((tick - h->gp.history_gossip) * v.rounds, 0);
    std::vector<int32_t> slot_last((size_t)v.ring);
    std::vector<uint32_t> mtopic((size_t)v.ring);
    hipError_t he = hipMemcpyAsync(slot_last.data(), v.slot_last, (size_t)v.ring * 4, hipMemcpyDeviceToHost, h->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(mtopic.data(), v.mtopic, (size_t)v.ring * 4, hipMemcpyDeviceToHost, h->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(h->stream);
    if (he != hipSuccess) return hip_check(h, he, "wire slot tables");
    std::vector<int32_t> cand_ptr((size_t)T + 1, 0);
    std::vector<uint16_t> cand;
    for (int32_t t = 0; t < T; ++t) {
        cand_ptr[(size_t)t] = (int32_t)cand.size();
        for (int32_t m = 0; m < v.ring; ++m)
            if (slot_last[(size_t)m] >= lo_round && (int32_t)mtopic[(size_t)m] == t) cand.push_back((uint16_t)m);
    }
    cand_ptr[(size_t)T] = (int32_t)cand.size();

    const int64_t npt = (int64_t)(p1 - p0) * T;
    uint32_t rp[2] = {0, 0};
    {
        he = hipMemcpyAsync(&rp[0], h->d_row_ptr + p0, 4, hipMemcpyDeviceToHost, h->stream);
        if (he == hipSuccess) he = hipMemcpyAsync(&rp[1], h->d_row_ptr + p1, 4, hipMemcpyDeviceToHost, h->stream);
        if (he == hipSuccess) he = hipStreamSynchronize(h->stream);
        if (he != hipSuccess) return hip_check(h, he, "wire row bounds");
    }
    const int64_t ne = (int64_t)rp[1] - rp[0];

    // device scratch (freed at the end of the call)
    std::vector<void*> bufs;
    auto alloc = [&](void** p, size_t n) {
        if (he == hipSuccess) he = hipMalloc(p, std::max<size_t>(n, 8));
        if (he == hipSuccess) bufs.push_back(*p);
    };
    WireArgs a{};
    uint8_t* d_names = nullptr;
    uint32_t* d_name_off = nullptr;
    uint8_t* d_pid = nullptr;
    uint16_t* d_cand = nullptr;
    int32_t* d_cand_ptr = nullptr;
    alloc((void**)&d_names, name_bytes.size());
    alloc((void**)&d_name_off, name_off.size() * 4);
    alloc((void**)&d_cand, cand.size() * 2);
    alloc((void**)&d_cand_ptr, cand_ptr.size() * 4);
    if (names->peer_id_len) alloc((void**)&d_pid, (size_t)h->n * names->peer_id_len);
    alloc((void**)&a.n_pt, (size_t)(npt + 1) * 8);
    alloc((void**)&a.id_off, (size_t)(npt + 1) * 8);
    alloc((void**)&a.rsize, (size_t)(ne + 1) * 8);
    alloc((void**)&a.rflag, (size_t)(ne + 1) * 4);
    alloc((void**)&a.roff, (size_t)(ne + 1) * 8);
    alloc((void**)&a.rcnt, (size_t)(ne + 1) * 4);
    alloc((void**)&a.err, 4);
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    auto finish = [&](int rc) {
        (void)hipStreamSynchronize(h->stream);
        for (void* p : bufs) (void)hipFree(p);
        if (tmp) (void)hipFree(tmp);
        return rc;
    };
    if (he != hipSuccess) return finish(hip_check(h, he, "wire scratch"));
    auto up = [&](void* d, const void* s, size_t n) {
        if (he == hipSuccess && n) he = hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, h->stream);
    };
    up(d_names, name_bytes.data(), name_bytes.size());
    up(d_name_off, name_off.data(), name_off.size() * 4);
    up(d_cand, cand.data(), cand.size() * 2);
    up(d_cand_ptr, cand_ptr.data(), cand_ptr.size() * 4);
    if (d_pid) up(d_pid, names->peer_ids, (size_t)h->n * names->peer_id_len);
    if (he == hipSuccess) he = hipMemsetAsync(a.n_pt, 0, (size_t)(npt + 1) * 8, h->stream);
    if (he == hipSuccess) he = hipMemsetAsync(a.rsize, 0, (size_t)(ne + 1) * 8, h->stream);
    if (he == hipSuccess) he = hipMemsetAsync(a.rflag, 0, (size_t)(ne + 1) * 4, h->stream);
    if (he == hipSuccess) he = hipMemsetAsync(a.err, 0, 4, h->stream);
    if (he != hipSuccess) return finish(hip_check(h, he, "wire tables"));

    a.row_ptr = h->d_row_ptr; a.col = h->d_col; a.rev = h->d_rev; a.owner = h->d_owner;
    a.ctl = extra_ctl(h);            // parity 0: the heartbeat's output
    a.gsel = v.gsel;
    a.smask = h->d_smask;
    a.cells = v.cells;
    a.N = h->n; a.E = h->e; a.T = T; a.R = v.rounds;
    a.mtopic = v.mtopic; a.morigin = v.morigin; a.minv = v.minv; a.mid = v.mid;
    a.cand = d_cand; a.cand_ptr = d_cand_ptr;
    a.g = g; a.lo_round = lo_round;
    a.p0 = p0; a.p1 = p1; a.e0 = rp[0]; a.e1 = rp[1];
    a.names = d_names; a.name_off = d_name_off;
    a.peer_ids = d_pid; a.pid_len = names->peer_id_len;
    a.backoff = names->prune_backoff_s;
    a.max_ihave = h->gp.max_ihave_length;
    a.out = d_out; a.refs = d_refs;
    a.unsub_backoff = (uint64_t)(h->gp.unsubscribe_backoff_ns / 1000000000);
    WirePx wp{};
    if (deliver_wire_px(h, &wp)) {                  // WithPeerExchange: the lists' inputs
        if (h->gp.prune_peers > kWirePxMax) {
            h->err = "PrunePeers above " + std::to_string(kWirePxMax) + ": PX lists are not encoded";
            return finish(GSIM_ERANGE);
        }
        a.rstate = h->d_rstate; a.sub = h->d_sub; a.pxs = wp.pxs; a.seed = wp.seed; a.tick = tick;
        a.prune_peers = h->gp.prune_peers; a.pxl = wp.pxl; a.pxl_tick = wp.pxl_tick; a.n_pxl = wp.n_pxl;
    }
    if (!a.ctl) return finish(GSIM_ESTATE);

    constexpr int B = 256;
    if (npt) hipLaunchKernelGGL(k_wire_ids_count, dim3((uint32_t)((npt + B - 1) / B)), dim3(B), 0, h->stream, a);
    if (ne) hipLaunchKernelGGL(k_wire_size, dim3((uint32_t)((ne + B - 1) / B)), dim3(B), 0, h->stream, a);
    int rc = hip_check(h, hipGetLastError(), "k_wire_size");
    // the scans (n + 1 entries each, the last input 0: its output is the total)
    if (!rc) rc = exclusive_scan(h, (const uint64_t*)a.n_pt, a.id_off, npt + 1, &tmp, &tmp_bytes);
    if (!rc) rc = exclusive_scan(h, (const uint64_t*)a.rsize, a.roff, ne + 1, &tmp, &tmp_bytes);
    if (!rc) rc = exclusive_scan(h, (const uint32_t*)a.rflag, a.rcnt, ne + 1, &tmp, &tmp_bytes);
    if (rc) return finish(rc);
    uint64_t tot_ids = 0, tot_bytes = 0;
    uint32_t tot_rpcs = 0, err = 0;
    he = hipMemcpyAsync(&tot_ids, a.id_off + npt, 8, hipMemcpyDeviceToHost, h->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(&tot_bytes, a.roff + ne, 8, hipMemcpyDeviceToHost, h->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(&tot_rpcs, a.rcnt + ne, 4, hipMemcpyDeviceToHost, h->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(&err, a.err, 4, hipMemcpyDeviceToHost, h->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(h->stream);
    if (he != hipSuccess) return finish(hip_check(h, he, "wire totals"));
    if (err & 1u) {
        h->err = "an IHAVE target without message ids in the gossip window";
        return finish(GSIM_ESTATE);
    }
    if (err & 2u) {
        h->err = "a gossip window holds more than MaxIHaveLength ids: emitGossip's per-target subsets are not encoded";
        return finish(GSIM_ESTATE);
    }

    *n_rpcs = tot_rpcs;
    *bytes = tot_bytes;
    if (tot_bytes > out_cap || (int64_t)tot_rpcs > ref_cap) {
        h->err = "wire output buffers too small";
        return finish(GSIM_ERANGE);
    }
    if ((tot_bytes && !d_out) || (tot_rpcs && !d_refs)) return finish(GSIM_EINVAL);
    alloc((void**)&a.ids, (size_t)tot_ids * 4);
    if (he != hipSuccess) return finish(hip_check(h, he, "wire id scratch"));
    if (npt) hipLaunchKernelGGL(k_wire_ids, dim3((uint32_t)((npt + B - 1) / B)), dim3(B), 0, h->stream, a);
    if (ne) hipLaunchKernelGGL(k_wire_write, dim3((uint32_t)((ne + B - 1) / B)), dim3(B), 0, h->stream, a);
    rc = hip_check(h, hipGetLastError(), "k_wire_write");
    return finish(rc);
}
