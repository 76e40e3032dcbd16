// shard.hip — graph-sharded networks over several GPUs (SURVEY.md §8(e),
// DESIGN.md §5): a group of shard handles and the halo exchange between them.
//
// The reference runs one router per host and moves RPCs between hosts over
// libp2p streams (gossipsub.go:1138-1202 sendRPC).  Here one simulated network
// is split into contiguous peer ranges (shard_plan.cpp).  Each shard is an
// ordinary engine handle over its local graph — owned rows plus ghost rows
// (a remote neighbour's connections into the shard) — that computes only for
// its owned peers.  Copies are pushed: a shard walks its own forwarders'
// whole rows and sends each copy to a ghost receiver to the receiver's shard
// as (the edge's index there, slot), which applies it (AcceptFrom, claim,
// records) before its commit (GSIM_SHARD_PULL=1: round 2's pull, where the
// receiver's shard walks the ghost forwarders' rows itself).  What moves:
//   per round      the copies to other shards' peers (push), and the
//                  forwarders of the round (peer, first sender, slot), from
//                  every shard to every other (the frontier: ghost cells);
//   per control    GRAFT/PRUNE records written into ghost receivers' inboxes,
//                  and then the router state of cross edges (mesh and fanout
//                  bits, connected, direct, publish gate) into ghost rows;
//   per heartbeat  the gossip marks of cross edges (emitGossip's choice per
//                  topic + the advertiser's IWANT gate), into ghost rows.
// A ghost's cell holds the first-seen round its shard exported, which is all
// IHAVE needs to know about a remote advertiser.  Two transports move the
// bytes: in-process (every shard in this process, one HIP stream each;
// device-to-device copies) and RCCL (one shard per process, ncclSend/ncclRecv
// grouped all-to-all over xGMI).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <tuple>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "gsim.h"
#include "gsim_internal.h"
#include "shard_layout.h"

using namespace gsim;

namespace {

// ---------------------------------------------------------------------------
// exchange kernels

constexpr uint32_t kNone = 0xFFFFFFFFu;

// local peer ranges of the shards ([lo[s], lo[s+1]) are shard s's peers)
struct PeerRanges {
    int64_t lo[GSIM_MAX_SHARDS + 1];
    int32_t K;
};

// GRAFT/PRUNE records written into ghost receivers' inboxes (plane `ctl`,
// summary `cany`), one thread per ghost peer with a summary bit: entries
// (owner shard's edge | topic << 32 | bits << 40) to the ghost's shard.  A
// block counts its entries per shard in LDS and reserves each shard's range
// with one atomic.
__global__ __launch_bounds__(256) void k_ctl_export(uint8_t* ctl, uint64_t* cany, const uint32_t* row_ptr,
                                                    const uint32_t* ymap, const uint64_t* smask, PeerRanges pr,
                                                    int64_t E, int32_t T,
                                                    int64_t olo, int64_t ohi, int64_t n, uint64_t* out,
                                                    uint32_t* cnt, int64_t cap)
{
    __shared__ uint32_t s_cnt[GSIM_MAX_SHARDS], s_base[GSIM_MAX_SHARDS];
    // a summary word may be a superset (all ones after an ABI write of the inbox)
    const uint64_t tmask = T >= 64 ? ~0ull : ((1ull << T) - 1);
    const int64_t nghost = olo + (n - ohi);
    const int tid = threadIdx.x;
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < nghost; b0 += (int64_t)gridDim.x * 256) {   // block-uniform
        for (int q = tid; q < pr.K; q += 256) s_cnt[q] = 0;
        __syncthreads();
        const int64_t x = b0 + tid;
        int64_t g = -1;
        uint64_t any = 0;
        uint32_t d = 0, mine = 0, off = 0;
        if (x < nghost) {
            g = x < olo ? x : ohi + (x - olo);
            any = cany[g] & tmask & smask_of(smask, (uint32_t)g);
            if (cany[g]) cany[g] = 0;
            while ((int32_t)d + 1 < pr.K && g >= pr.lo[d + 1]) ++d;
            for (uint64_t r = any; r; r &= r - 1) {
                const int32_t t = __ffsll((long long)r) - 1;
                const int64_t pl = slot_idx(smask_of(smask, (uint32_t)g), t, E, 0);
                for (uint32_t e = row_ptr[g]; e < row_ptr[g + 1]; ++e) mine += ctl[pl + e] != 0;
            }
            if (mine) off = atomicAdd(&s_cnt[d], mine);
        }
        __syncthreads();
        for (int q = tid; q < pr.K; q += 256) s_base[q] = s_cnt[q] ? atomicAdd(cnt + q, s_cnt[q]) : 0u;
        __syncthreads();
        if (mine) {
            int64_t pos = (int64_t)s_base[d] + off;
            for (uint64_t r = any; r; r &= r - 1) {
                const int32_t t = __ffsll((long long)r) - 1;
                const int64_t pl = slot_idx(smask_of(smask, (uint32_t)g), t, E, 0);
                for (uint32_t e = row_ptr[g]; e < row_ptr[g + 1]; ++e) {
                    const int64_t i = pl + e;
                    const uint8_t c = ctl[i];
                    if (!c) continue;
                    ctl[i] = 0;
                    if (pos < cap) out[(int64_t)d * cap + pos] = (uint64_t)ymap[e] | ((uint64_t)t << 32) | ((uint64_t)c << 40);
                    ++pos;
                }
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_ctl_import(const uint64_t* in, int64_t n_in, uint8_t* ctl, uint64_t* cany,
                                                    const uint32_t* owner, const uint64_t* smask, int64_t E)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n_in; x += stride) {
        const uint64_t v = in[x];
        const uint32_t e = (uint32_t)v;
        const int32_t t = (int32_t)((v >> 32) & 0xFF);
        const uint8_t bits = (uint8_t)(v >> 40);
        const uint64_t m = smask_of(smask, owner[e]);
        if (!slot_has(m, t)) continue;
        uint8_t* p = ctl + slot_idx(m, t, E, e);
        *p = (uint8_t)(*p | bits);      // one entry per (receiver edge, topic)
        atomicOr(reinterpret_cast<unsigned long long*>(cany + owner[e]), 1ull << t);
    }
}

// emitGossip's choices of the owned rows' cross edges, one topic mask per
// edge in cross-out order, with the advertiser's IWANT gate (gstate).
__global__ __launch_bounds__(256) void k_gsel_export(const uint32_t* xgather, int64_t n_cross, const uint8_t* gsel,
                                                     const uint8_t* gstate, const uint32_t* owner, const uint64_t* smask,
                                                     int32_t T, int64_t E, uint64_t* out, uint8_t* gs_out)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n_cross; q += stride) {
        const uint32_t e = xgather[q];
        uint64_t m = 0;
        const uint64_t sm = smask_of(smask, owner[e]);
        for (int32_t t = 0; t < T; ++t)
            if (slot_has(sm, t)) m |= (uint64_t)(gsel[slot_idx(sm, t, E, e)] != 0) << t;
        out[q] = m;
        gs_out[q] = gstate[e];
    }
}

// The same in edge order: each owned-row edge reads its topic planes where
// they lie (neighbouring lanes, neighbouring bytes) and a cross edge stores its
// mask at its cross-out index (xpos).  In cross-out order every plane read was
// a random byte gather: 16 lines per cross edge at C3 (0.33 ms per shard and
// tick at K = 8; with k_holder_import's batched loads, the mean shard 11.95 -> 11.86 ms,
// gpurun_out/r05x_s8).
__global__ __launch_bounds__(256) void k_gsel_export_e(const uint32_t* xpos, int64_t e_lo, int64_t e_hi,
                                                       const uint8_t* gsel, const uint8_t* gstate, const uint32_t* owner,
                                                       const uint64_t* smask, int32_t T, int64_t E, uint64_t* out,
                                                       uint8_t* gs_out)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = e_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e_hi; e += stride) {
        const uint32_t q = xpos[e];
        if (q == 0xFFFFFFFFu) continue;
        uint64_t m = 0;
        const uint64_t sm = smask_of(smask, owner[e]);
        for (int32_t t = 0; t < T; ++t)
            if (slot_has(sm, t)) m |= (uint64_t)(gsel[slot_idx(sm, t, E, e)] != 0) << t;
        out[q] = m;
        gs_out[q] = gstate[e];
    }
}

// ... into the ghost rows: every topic plane of every ghost-row edge.
__global__ __launch_bounds__(256) void k_gsel_import(const uint64_t* in, const uint8_t* gs_in, uint8_t* gsel,
                                                     uint8_t* gstate, const uint32_t* owner, const uint64_t* smask,
                                                     int32_t T, int64_t E, int64_t e_lo, int64_t e_hi)
{
    const int64_t nghost = e_lo + (E - e_hi);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < nghost; x += stride) {
        const int64_t e = x < e_lo ? x : e_hi + (x - e_lo);
        const uint64_t m = in[e];
        const uint64_t sm = smask_of(smask, owner[e]);
        for (int32_t t = 0; t < T; ++t)
            if (slot_has(sm, t)) gsel[slot_idx(sm, t, E, e)] = (uint8_t)((m >> t) & 1ull);
        gstate[e] = gs_in[e];
    }
}

// The router state of the owned rows' cross edges (cross-out order): the
// mesh and fanout bits per topic, connected | direct | publish gate.
__global__ __launch_bounds__(256) void k_router_export(const uint32_t* xgather, int64_t n_cross, const uint8_t* mflags,
                                                       const uint8_t* rstate, const uint8_t* direct, const double* score,
                                                       const uint32_t* rev, const uint32_t* owner, const uint64_t* smask,
                                                       double pub_thr, int32_t T, int64_t E,
                                                       uint64_t* mesh, uint64_t* fan, uint8_t* flags)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n_cross; q += stride) {
        const uint32_t e = xgather[q];
        uint64_t mm = 0, fm = 0;
        const uint64_t sm = smask_of(smask, owner[e]);
        for (int32_t t = 0; t < T; ++t) {
            if (!slot_has(sm, t)) continue;
            const uint8_t f = mflags[slot_idx(sm, t, E, e)];
            mm |= (uint64_t)((f & GSIM_TF_MESH) != 0) << t;
            fm |= (uint64_t)((f & GSIM_TF_FANOUT) != 0) << t;
        }
        mesh[q] = mm;
        fan[q] = fm;
        flags[q] = (uint8_t)(((rstate[e] & GSIM_ES_CONNECTED) ? 1 : 0) | (direct[e] ? 2 : 0) |
                             (score[rev[e]] >= pub_thr ? 4 : 0));
    }
}

// ... into the ghost rows (the ghost's edges into this shard), and the
// delivery's mesh masks of the ghost rows of at most 64 connections (zeroed
// before: bit (row position) per topic with the mesh bit or a direct peer).
__global__ __launch_bounds__(256) void k_router_import(const uint64_t* mesh, const uint64_t* fan, const uint8_t* flags,
                                                       uint8_t* mflags, uint8_t* rstate, uint8_t* direct, uint8_t* pgate,
                                                       int32_t T, int64_t E, int64_t e_lo, int64_t e_hi,
                                                       const uint32_t* row_ptr, const uint32_t* owner, int64_t n,
                                                       uint64_t* mmask, const uint64_t* smask)
{
    const int64_t nghost = e_lo + (E - e_hi);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < nghost; x += stride) {
        const int64_t e = x < e_lo ? x : e_hi + (x - e_lo);
        const uint64_t mm = mesh[e], fm = fan[e];
        const uint64_t sm = smask_of(smask, owner[e]);
        for (int32_t t = 0; t < T; ++t)
            if (slot_has(sm, t))
                mflags[slot_idx(sm, t, E, e)] = (uint8_t)((((mm >> t) & 1ull) ? GSIM_TF_MESH : 0) |
                                                          (((fm >> t) & 1ull) ? GSIM_TF_FANOUT : 0));
        const uint8_t f = flags[e];
        rstate[e] = (f & 1) ? GSIM_ES_CONNECTED : 0;
        direct[e] = (f & 2) ? 1 : 0;
        pgate[e] = (f & 4) ? 1 : 0;
        if (mmask) {
            const uint32_t r = owner[e], b = row_ptr[r];
            if (row_ptr[r + 1] - b <= 64u) {
                const uint64_t bit = 1ull << (e - b);
                for (uint64_t q = (f & 2) ? (T >= 64 ? ~0ull : (1ull << T) - 1) : mm; q; q &= q - 1)
                    atomicOr(reinterpret_cast<unsigned long long*>(mmask + (int64_t)(__ffsll((long long)q) - 1) * n + r), bit);
            }
        }
    }
}

// zero the ghost rows' masks of every topic
__global__ __launch_bounds__(256) void k_ghost_mask_clear(uint64_t* mmask, int64_t olo, int64_t ohi, int64_t n,
                                                          int32_t T)
{
    const int64_t nghost = olo + (n - ohi);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < nghost * T; x += stride) {
        const int64_t t = x / nghost, y = x - t * nghost;
        mmask[t * n + (y < olo ? y : ohi + (y - olo))] = 0;
    }
}

// Control-round mesh changes of other shards' cross edges, into this shard's
// ghost rows (router flags and the delivery's mesh masks).
struct EdgeBases {
    int64_t b[GSIM_MAX_SHARDS];
};

__global__ __launch_bounds__(256) void k_router_delta(const uint64_t* in, int64_t n_in, int32_t self, EdgeBases gb,
                                                      uint8_t* mflags, const uint8_t* direct, const uint32_t* row_ptr,
                                                      const uint32_t* owner, const uint64_t* smask, int64_t E, int64_t n,
                                                      uint64_t* mmask)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n_in; x += stride) {
        const uint64_t v = in[x];
        if ((int32_t)((v >> 6) & 63) != self) continue;
        const int32_t src = (int32_t)(v & 63), t = (int32_t)((v >> 12) & 0xFF);
        const uint8_t fl = (uint8_t)((v >> 20) & 0xFF);
        const int64_t ge = gb.b[src] + (int64_t)(v >> 32);
        const uint64_t sm = smask_of(smask, owner[ge]);
        if (!slot_has(sm, t)) continue;
        uint8_t* p = mflags + slot_idx(sm, t, E, ge);
        *p = (uint8_t)((*p & ~(GSIM_TF_MESH | GSIM_TF_FANOUT)) | fl);
        if (mmask) {
            const uint32_t r = owner[ge], b = row_ptr[r];
            if (row_ptr[r + 1] - b <= 64u) {
                const uint64_t bit = 1ull << (ge - b);
                unsigned long long* w = reinterpret_cast<unsigned long long*>(mmask + (int64_t)t * n + r);
                if (fl & GSIM_TF_MESH) atomicOr(w, bit);
                else if (!direct[ge]) atomicAnd(w, ~bit);
            }
        }
    }
}

// Copy push: an owned-row cross edge's index at the
// receiver's shard = that shard's ghost block of this shard's peers (rb) +
// the edge's position in the cross-out list to it.
__global__ __launch_bounds__(256) void k_xre_build(const uint32_t* xq, const uint32_t* col, const uint8_t* pshard,
                                                   EdgeBases rb, uint32_t* xre, int64_t E)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride)
        xre[e] = xq[e] == 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)(rb.b[pshard[col[e]]] + (int64_t)xq[e]);
}

int grid_for(int64_t n)
{
    int64_t g = (n + 255) / 256;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, 16384));
}

// ---------------------------------------------------------------------------
// transports

enum { DT_U32 = 0, DT_I32 = 1, DT_U64 = 2 };
enum { OP_SUM = 0, OP_MAX = 1 };

struct Transport {
    virtual ~Transport() = default;
    // send[l][d]: 64-bit values local shard l sends shard d -> recv[l][s]
    virtual int exchange_counts(const std::vector<std::vector<uint64_t>>& send,
                                std::vector<std::vector<uint64_t>>& recv) = 0;
    // bytes sp[l][d] (sb[l][d] of them) from local shard l to shard d, landing
    // at d's rp[.][l] (rb bytes)
    virtual int alltoallv(const std::vector<std::vector<const void*>>& sp, const std::vector<std::vector<uint64_t>>& sb,
                          const std::vector<std::vector<void*>>& rp, const std::vector<std::vector<uint64_t>>& rb) = 0;
    // elementwise over every shard's array p[l] (count elements), in place
    virtual int allreduce(const std::vector<void*>& p, int64_t count, int dt, int op) = 0;
    // shard s's block (bytes[s] at byte offset off[s]) into every shard's buf
    virtual int allgatherv(const std::vector<void*>& buf, const std::vector<uint64_t>& off,
                           const std::vector<uint64_t>& bytes) = 0;
    virtual int sync() = 0;
    std::string err;
};

// Every shard in this process (possibly on one device): device-to-device
// copies between the shards' buffers, ordered by synchronizing the streams.
struct LocalTransport : Transport {
    std::vector<gsim_handle*> hs;   // index = shard id
    int sync() override
    {
        for (gsim_handle* h : hs) {
            (void)hipSetDevice(h->device);
            if (hipStreamSynchronize(h->stream) != hipSuccess) { err = "stream synchronize"; return GSIM_EDEVICE; }
        }
        return GSIM_OK;
    }
    int exchange_counts(const std::vector<std::vector<uint64_t>>& send, std::vector<std::vector<uint64_t>>& recv) override
    {
        const size_t K = hs.size();
        recv.assign(K, std::vector<uint64_t>(K, 0));
        for (size_t a = 0; a < K; ++a)
            for (size_t b = 0; b < K; ++b) recv[b][a] = send[a][b];
        return GSIM_OK;
    }
    int alltoallv(const std::vector<std::vector<const void*>>& sp, const std::vector<std::vector<uint64_t>>& sb,
                  const std::vector<std::vector<void*>>& rp, const std::vector<std::vector<uint64_t>>& rb) override
    {
        int rc = sync();
        if (rc) return rc;
        const size_t K = hs.size();
        for (size_t a = 0; a < K; ++a)
            for (size_t b = 0; b < K; ++b) {
                if (a == b || !sb[a][b]) continue;
                if (rb[b][a] != sb[a][b]) { err = "exchange size mismatch"; return GSIM_EINVAL; }
                (void)hipSetDevice(hs[b]->device);
                if (hipMemcpyAsync(rp[b][a], sp[a][b], sb[a][b], hipMemcpyDefault, hs[b]->stream) != hipSuccess) {
                    err = "device copy";
                    return GSIM_EDEVICE;
                }
            }
        return sync();
    }
    int allreduce(const std::vector<void*>& p, int64_t count, int dt, int op) override
    {
        int rc = sync();
        if (rc) return rc;
        const size_t es = dt == DT_U64 ? 8 : 4, K = hs.size();
        std::vector<std::vector<uint8_t>> host(K, std::vector<uint8_t>(es * (size_t)count));
        for (size_t s = 0; s < K; ++s) {
            (void)hipSetDevice(hs[s]->device);
            if (hipMemcpy(host[s].data(), p[s], es * (size_t)count, hipMemcpyDeviceToHost) != hipSuccess) {
                err = "reduce readback";
                return GSIM_EDEVICE;
            }
        }
        std::vector<uint8_t> acc = host[0];
        for (size_t s = 1; s < K; ++s)
            for (int64_t i = 0; i < count; ++i) {
                if (dt == DT_U64) {
                    uint64_t& x = reinterpret_cast<uint64_t*>(acc.data())[i];
                    const uint64_t y = reinterpret_cast<const uint64_t*>(host[s].data())[i];
                    x = op == OP_SUM ? x + y : std::max(x, y);
                } else if (dt == DT_U32) {
                    uint32_t& x = reinterpret_cast<uint32_t*>(acc.data())[i];
                    const uint32_t y = reinterpret_cast<const uint32_t*>(host[s].data())[i];
                    x = op == OP_SUM ? x + y : std::max(x, y);
                } else {
                    int32_t& x = reinterpret_cast<int32_t*>(acc.data())[i];
                    const int32_t y = reinterpret_cast<const int32_t*>(host[s].data())[i];
                    x = op == OP_SUM ? x + y : std::max(x, y);
                }
            }
        for (size_t s = 0; s < K; ++s) {
            (void)hipSetDevice(hs[s]->device);
            if (hipMemcpy(p[s], acc.data(), es * (size_t)count, hipMemcpyHostToDevice) != hipSuccess) {
                err = "reduce upload";
                return GSIM_EDEVICE;
            }
        }
        return GSIM_OK;
    }
    int allgatherv(const std::vector<void*>& buf, const std::vector<uint64_t>& off,
                   const std::vector<uint64_t>& bytes) override
    {
        int rc = sync();
        if (rc) return rc;
        const size_t K = hs.size();
        for (size_t s = 0; s < K; ++s)
            for (size_t d = 0; d < K; ++d) {
                if (s == d || !bytes[s]) continue;
                (void)hipSetDevice(hs[d]->device);
                if (hipMemcpyAsync((uint8_t*)buf[d] + off[s], (const uint8_t*)buf[s] + off[s], bytes[s],
                                   hipMemcpyDefault, hs[d]->stream) != hipSuccess) {
                    err = "device copy";
                    return GSIM_EDEVICE;
                }
            }
        return sync();
    }
};

// One shard per process, RCCL over xGMI: every collective is enqueued on the
// shard's own stream, so the kernels before and after it stay stream-ordered.
struct RcclTransport : Transport {
    gsim_handle* h = nullptr;
    int k = 0, K = 1;
    ncclComm_t comm = nullptr;
    uint64_t* d_cnt = nullptr;     // [K*K] count matrix
    uint64_t* h_cnt = nullptr;     // pinned
    ~RcclTransport() override
    {
        if (d_cnt) (void)hipFree(d_cnt);
        if (h_cnt) (void)hipHostFree(h_cnt);
        if (comm) ncclCommDestroy(comm);
    }
    int check(ncclResult_t r, const char* what)
    {
        if (r == ncclSuccess) return GSIM_OK;
        err = std::string(what) + ": " + ncclGetErrorString(r);
        return GSIM_EDEVICE;
    }
    int sync() override
    {
        if (hipStreamSynchronize(h->stream) != hipSuccess) { err = "stream synchronize"; return GSIM_EDEVICE; }
        return GSIM_OK;
    }
    int exchange_counts(const std::vector<std::vector<uint64_t>>& send, std::vector<std::vector<uint64_t>>& recv) override
    {
        for (int d = 0; d < K; ++d) h_cnt[(size_t)k * K + d] = send[0][(size_t)d];
        if (hipMemcpyAsync(d_cnt + (size_t)k * K, h_cnt + (size_t)k * K, sizeof(uint64_t) * K, hipMemcpyHostToDevice,
                           h->stream) != hipSuccess) { err = "count upload"; return GSIM_EDEVICE; }
        int rc = check(ncclAllGather(d_cnt + (size_t)k * K, d_cnt, (size_t)K, ncclUint64, comm, h->stream),
                       "ncclAllGather(counts)");
        if (rc) return rc;
        if (hipMemcpyAsync(h_cnt, d_cnt, sizeof(uint64_t) * K * K, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
            { err = "count readback"; return GSIM_EDEVICE; }
        rc = sync();
        if (rc) return rc;
        recv.assign(1, std::vector<uint64_t>((size_t)K, 0));
        for (int s = 0; s < K; ++s) recv[0][(size_t)s] = h_cnt[(size_t)s * K + k];
        return GSIM_OK;
    }
    int alltoallv(const std::vector<std::vector<const void*>>& sp, const std::vector<std::vector<uint64_t>>& sb,
                  const std::vector<std::vector<void*>>& rp, const std::vector<std::vector<uint64_t>>& rb) override
    {
        int rc = check(ncclGroupStart(), "ncclGroupStart");
        for (int d = 0; d < K && !rc; ++d) {
            if (d == k) continue;
            if (sb[0][(size_t)d])
                rc = check(ncclSend(sp[0][(size_t)d], sb[0][(size_t)d], ncclChar, d, comm, h->stream), "ncclSend");
            if (!rc && rb[0][(size_t)d])
                rc = check(ncclRecv(rp[0][(size_t)d], rb[0][(size_t)d], ncclChar, d, comm, h->stream), "ncclRecv");
        }
        const int rc2 = check(ncclGroupEnd(), "ncclGroupEnd");
        return rc ? rc : rc2;
    }
    int allreduce(const std::vector<void*>& p, int64_t count, int dt, int op) override
    {
        const ncclDataType_t t = dt == DT_U64 ? ncclUint64 : dt == DT_U32 ? ncclUint32 : ncclInt32;
        return check(ncclAllReduce(p[0], p[0], (size_t)count, t, op == OP_SUM ? ncclSum : ncclMax, comm, h->stream),
                     "ncclAllReduce");
    }
    int allgatherv(const std::vector<void*>& buf, const std::vector<uint64_t>& off,
                   const std::vector<uint64_t>& bytes) override
    {
        int rc = check(ncclGroupStart(), "ncclGroupStart");
        for (int s = 0; s < K && !rc; ++s) {
            if (!bytes[(size_t)s]) continue;
            void* p = (uint8_t*)buf[0] + off[(size_t)s];
            rc = check(ncclBroadcast(p, p, bytes[(size_t)s], ncclChar, s, comm, h->stream), "ncclBroadcast");
        }
        const int rc2 = check(ncclGroupEnd(), "ncclGroupEnd");
        return rc ? rc : rc2;
    }
};

// One shard per process, exchanges through the caller's host collectives
// (gsim_host_transport): every device buffer is staged through pinned host
// memory.  Same call sequence as RcclTransport, so it runs the one-shard-
// per-process path of the group on any number of ranks per GPU.
struct HostTransport : Transport {
    gsim_handle* h = nullptr;
    int k = 0, K = 1;
    gsim_host_transport cb{};
    uint8_t* hs_ = nullptr;          // pinned staging: send | recv
    size_t hcap = 0;
    ~HostTransport() override
    {
        if (hs_) (void)hipHostFree(hs_);
    }
    int stage(size_t need)
    {
        if (need <= hcap) return GSIM_OK;
        if (hs_) (void)hipHostFree(hs_);
        hs_ = nullptr;
        hcap = 0;
        const size_t c = std::max<size_t>(need + need / 2, 1 << 16);
        if (hipHostMalloc((void**)&hs_, c, 0) != hipSuccess) { err = "pinned staging"; return GSIM_ENOMEM; }
        hcap = c;
        return GSIM_OK;
    }
    int sync() override
    {
        if (hipStreamSynchronize(h->stream) != hipSuccess) { err = "stream synchronize"; return GSIM_EDEVICE; }
        return GSIM_OK;
    }
    // host-to-host all-to-all of byte blocks (the rank's own block skipped)
    int a2a(const uint8_t* send, const std::vector<uint64_t>& sb, uint8_t* recv, const std::vector<uint64_t>& rb)
    {
        std::vector<uint64_t> sd((size_t)K, 0), rd((size_t)K, 0);
        for (int q = 1; q < K; ++q) { sd[(size_t)q] = sd[(size_t)q - 1] + sb[(size_t)q - 1]; rd[(size_t)q] = rd[(size_t)q - 1] + rb[(size_t)q - 1]; }
        if (cb.alltoallv(cb.ctx, send, sb.data(), sd.data(), recv, rb.data(), rd.data()) != 0) {
            err = "host alltoallv callback";
            return GSIM_EDEVICE;
        }
        return GSIM_OK;
    }
    int exchange_counts(const std::vector<std::vector<uint64_t>>& send, std::vector<std::vector<uint64_t>>& recv) override
    {
        // blocks are packed in rank order without this rank's own
        std::vector<uint64_t> out, in((size_t)K, 0), b((size_t)K, 8);
        for (int d = 0; d < K; ++d)
            if (d != k) out.push_back(send[0][(size_t)d]);
        out.push_back(0);
        b[(size_t)k] = 0;
        int rc = a2a(reinterpret_cast<const uint8_t*>(out.data()), b, reinterpret_cast<uint8_t*>(in.data()), b);
        if (rc) return rc;
        // the packed blocks skip this rank: unpack in rank order
        recv.assign(1, std::vector<uint64_t>((size_t)K, 0));
        size_t x = 0;
        for (int s = 0; s < K; ++s) {
            if (s == k) { recv[0][(size_t)s] = send[0][(size_t)s]; continue; }
            recv[0][(size_t)s] = in[x++];
        }
        return GSIM_OK;
    }
    int alltoallv(const std::vector<std::vector<const void*>>& sp, const std::vector<std::vector<uint64_t>>& sb,
                  const std::vector<std::vector<void*>>& rp, const std::vector<std::vector<uint64_t>>& rb) override
    {
        std::vector<uint64_t> s8((size_t)K, 0), r8((size_t)K, 0);
        size_t st = 0, rt = 0;
        for (int q = 0; q < K; ++q) {
            if (q == k) continue;
            s8[(size_t)q] = sb[0][(size_t)q];
            r8[(size_t)q] = rb[0][(size_t)q];
            st += s8[(size_t)q];
            rt += r8[(size_t)q];
        }
        int rc = stage(st + rt);
        if (rc) return rc;
        uint8_t* sh = hs_;
        uint8_t* rh = hs_ + st;
        size_t off = 0;
        for (int q = 0; q < K; ++q) {
            if (!s8[(size_t)q]) continue;
            if (hipMemcpyAsync(sh + off, sp[0][(size_t)q], s8[(size_t)q], hipMemcpyDeviceToHost, h->stream) != hipSuccess)
                { err = "staging download"; return GSIM_EDEVICE; }
            off += s8[(size_t)q];
        }
        if ((rc = sync())) return rc;
        if ((rc = a2a(sh, s8, rh, r8))) return rc;
        off = 0;
        for (int q = 0; q < K; ++q) {
            if (!r8[(size_t)q]) continue;
            if (hipMemcpyAsync(rp[0][(size_t)q], rh + off, r8[(size_t)q], hipMemcpyHostToDevice, h->stream) != hipSuccess)
                { err = "staging upload"; return GSIM_EDEVICE; }
            off += r8[(size_t)q];
        }
        return sync();            // the staging buffer is reused by the next exchange
    }
    int allreduce(const std::vector<void*>& p, int64_t count, int dt, int op) override
    {
        const size_t bytes = (size_t)count * (dt == DT_U64 ? 8 : 4);
        int rc = stage(bytes);
        if (rc) return rc;
        if (hipMemcpyAsync(hs_, p[0], bytes, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
            { err = "staging download"; return GSIM_EDEVICE; }
        if ((rc = sync())) return rc;
        if (cb.allreduce(cb.ctx, hs_, count, dt, op) != 0) { err = "host allreduce callback"; return GSIM_EDEVICE; }
        if (hipMemcpyAsync(p[0], hs_, bytes, hipMemcpyHostToDevice, h->stream) != hipSuccess)
            { err = "staging upload"; return GSIM_EDEVICE; }
        return sync();
    }
    int allgatherv(const std::vector<void*>& buf, const std::vector<uint64_t>& off,
                   const std::vector<uint64_t>& bytes) override
    {
        // this rank's block to every other rank, theirs into their offsets
        std::vector<std::vector<const void*>> sp(1, std::vector<const void*>((size_t)K, nullptr));
        std::vector<std::vector<void*>> rp(1, std::vector<void*>((size_t)K, nullptr));
        std::vector<std::vector<uint64_t>> sb(1, std::vector<uint64_t>((size_t)K, 0)), rb = sb;
        for (int q = 0; q < K; ++q) {
            if (q == k) continue;
            sp[0][(size_t)q] = (const uint8_t*)buf[0] + off[(size_t)k];
            sb[0][(size_t)q] = bytes[(size_t)k];
            rp[0][(size_t)q] = (uint8_t*)buf[0] + off[(size_t)q];
            rb[0][(size_t)q] = bytes[(size_t)q];
        }
        return alltoallv(sp, sb, rp, rb);
    }
};

}  // namespace

// ---------------------------------------------------------------------------
// the group

struct gsim_group {
    int K = 1;
    std::vector<gsim_handle*> hs;     // local shards
    std::vector<int> ids;             // their shard ids
    std::unique_ptr<Transport> tr;
    std::string err;
    std::vector<int64_t> bounds;
    int64_t N = 0, E = 0;
    std::vector<std::vector<uint32_t>> gid;   // per local shard: local -> global peer id (host)
    std::vector<std::vector<uint64_t>> gidx;  // per local shard: local -> global edge index (host)
    std::vector<uint64_t> sub;                // the peers' subscriptions (publish: fanout possible?)
    std::vector<uint32_t> row_ptr;            // the global CSR rows (group readback: a range's global edges)
    int32_t ring = 0, rounds = 0;
    bool msgs = false;
    bool router_dirty = true;                 // ghost rows' router state must be re-imported
    uint32_t xseq = 0;                        // exchanges so far (the tag's sequence part, tagged_counts)
    // GSIM_GROUP_SERIAL=1: each shard's work completes before the next
    // shard's starts (in-process groups on one device: per-shard kernel
    // times as if each shard had the device to itself)
    bool serial = false;

    void settle(gsim_handle* h)
    {
        if (serial) (void)hipStreamSynchronize(h->stream);
    }

    int fail(int rc, const std::string& m)
    {
        err = m;
        return rc;
    }
    int take(gsim_handle* h, int rc)   // adopt a shard's error message
    {
        if (rc) err = "shard: " + h->err;
        return rc;
    }
    int take_tr(int rc)
    {
        if (rc) err = "exchange: " + tr->err;
        return rc;
    }
};

namespace {

template <typename T>
int dalloc(gsim_handle* h, T** p, size_t n)
{
    *p = nullptr;
    hipError_t e = hipMalloc((void**)p, sizeof(T) * std::max<size_t>(n, 1));
    if (e != hipSuccess) { h->err = std::string("hipMalloc: ") + hipGetErrorString(e); return GSIM_ENOMEM; }
    h->bytes_allocated += sizeof(T) * n;
    return GSIM_OK;
}

void free_shard_bufs(ShardCtx* s)
{
    auto f = [](void* p) { if (p) (void)hipFree(p); };
    f(s->d_gid); f(s->d_g2l); f(s->d_sptr); f(s->d_sedge); f(s->d_xq); f(s->d_rdel); f(s->d_rdel_n); f(s->d_rdel_in); f(s->d_ymap); f(s->d_xgather); f(s->d_xpos); f(s->d_pgate);
    f(s->d_fout); f(s->d_fcnt); f(s->d_fin); f(s->d_cout); f(s->d_ccnt); f(s->d_cin);
    f(s->d_rmesh_out); f(s->d_rfan_out); f(s->d_rflag_out); f(s->d_rmesh_in); f(s->d_rfan_in); f(s->d_rflag_in);
    f(s->d_gout); f(s->d_gsout); f(s->d_gin); f(s->d_gsin);
    f(s->d_xre); f(s->d_pshard); f(s->d_xwo); f(s->d_xwq); f(s->d_xbits); f(s->d_xsend); f(s->d_xrecv); f(s->d_xn);
    f(s->d_xsrc); f(s->d_hbits); f(s->d_hslots); f(s->d_hsend); f(s->d_hn); f(s->d_hsrc);
    if (s->h_xsrc) (void)hipHostFree(s->h_xsrc);
    if (s->h_hsrc) (void)hipHostFree(s->h_hsrc);
    f(s->d_pxout); f(s->d_pxcnt); f(s->d_pxin);
    if (s->h_counts) (void)hipHostFree(s->h_counts);
    if (s->h_xcnt) (void)hipHostFree(s->h_xcnt);
    ShardCtx fresh;
    fresh.k = s->k;
    fresh.K = s->K;
    fresh.push = s->push;
    *s = fresh;
}

void free_shard_ctx(gsim_handle* h)
{
    if (!h->sh) return;
    free_shard_bufs(h->sh);
    delete h->sh;
    h->sh = nullptr;
}

// grow a device buffer (contents are not kept)
template <typename T>
int ensure(gsim_handle* h, T** p, int64_t* cap, int64_t need)
{
    if (*cap >= need && *p) return GSIM_OK;
    if (*p) { (void)hipStreamSynchronize(h->stream); (void)hipFree(*p); *p = nullptr; }
    const int64_t c = std::max<int64_t>(need, 1) + need / 4;
    int rc = dalloc(h, p, (size_t)c);
    *cap = rc ? 0 : c;
    return rc;
}

int sync_all(gsim_group* g)
{
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        if (hipStreamSynchronize(h->stream) != hipSuccess) return g->fail(GSIM_EDEVICE, "stream synchronize");
    }
    return GSIM_OK;
}

// Exchange kinds, the high part of a count's tag (tagged_counts).
enum { XK_DENSE = 1, XK_CONTROL, XK_RDELTA, XK_FRONTIER, XK_COPIES, XK_GBASE, XK_PX, XK_PXA };
constexpr int kCountBits = 48;
constexpr uint64_t kCountMask = (1ull << kCountBits) - 1;

// The count exchange in front of every payload exchange, with a symmetry
// check.  Each 64-bit count carries a 16-bit tag in its top bits: the
// exchange kind and the group's running exchange number.  Every process runs
// the same sequence of exchanges, so a shard that receives another kind or
// number -- its peer's control flow went another way -- or a count other
// than the one it expects (`expect`, when the receiving side knows its size
// itself, as the dense exchanges do) returns GSIM_ESTATE before any payload
// moves.  Without the check such a mismatch reaches the payload collective:
// gloo aborts on the size ("38576 vs 0") and RCCL's ncclRecv
// waits forever.
int tagged_counts(gsim_group* g, int kind, const std::vector<std::vector<uint64_t>>& scnt,
                  std::vector<std::vector<uint64_t>>& rcnt, const std::vector<std::vector<uint64_t>>* expect = nullptr)
{
    const uint64_t tag = ((uint64_t)(kind & 0xF) << 12 | (g->xseq & 0xFFF)) << kCountBits;
    ++g->xseq;
    std::vector<std::vector<uint64_t>> t = scnt;
    for (auto& row : t)
        for (uint64_t& c : row) {
            if (c > kCountMask) return g->fail(GSIM_ERANGE, "exchange count over 2^48");
            c |= tag;
        }
    int rc = g->take_tr(g->tr->exchange_counts(t, rcnt));
    if (rc) return rc;
    for (size_t l = 0; l < rcnt.size(); ++l)
        for (size_t q = 0; q < rcnt[l].size(); ++q) {
            const uint64_t got = rcnt[l][q];
            if ((got & ~kCountMask) != tag)
                return g->fail(GSIM_ESTATE, "exchange sequence mismatch: shard " + std::to_string(q) + " sent kind " +
                                                std::to_string((got >> (kCountBits + 12)) & 0xF) + " #" +
                                                std::to_string((got >> kCountBits) & 0xFFF) + ", shard " +
                                                std::to_string(g->ids[l]) + " expects kind " + std::to_string(kind) +
                                                " #" + std::to_string((tag >> kCountBits) & 0xFFF));
            rcnt[l][q] = got & kCountMask;
            if (expect && (int)q != g->ids[l] && rcnt[l][q] != (*expect)[l][q])
                return g->fail(GSIM_ESTATE, "exchange size mismatch: shard " + std::to_string(q) + " sends " +
                                                std::to_string(rcnt[l][q]) + " B, shard " + std::to_string(g->ids[l]) +
                                                " expects " + std::to_string((*expect)[l][q]) + " B");
        }
    return GSIM_OK;
}

// A dense exchange over the cross edges: every local shard's cross-out
// ordered `elem`-byte records (out[l] at xoff) into the other shards' ghost
// blocks (in[l] at gbase).  Both sides know the sizes from the layout; the
// tagged count exchange checks that they agree before the payload moves.
int exchange_dense(gsim_group* g, const std::vector<const void*>& out, const std::vector<void*>& in, size_t elem)
{
    const size_t L = g->hs.size();
    const int K = g->K;
    std::vector<std::vector<const void*>> sp(L, std::vector<const void*>((size_t)K, nullptr));
    std::vector<std::vector<void*>> rp(L, std::vector<void*>((size_t)K, nullptr));
    std::vector<std::vector<uint64_t>> sb(L, std::vector<uint64_t>((size_t)K, 0)), rb = sb;
    for (size_t l = 0; l < L; ++l) {
        const ShardCtx* s = g->hs[l]->sh;
        for (int q = 0; q < K; ++q) {
            sp[l][(size_t)q] = (const uint8_t*)out[l] + (size_t)s->xoff[(size_t)q] * elem;
            sb[l][(size_t)q] = (uint64_t)(s->xoff[(size_t)q + 1] - s->xoff[(size_t)q]) * elem;
            rp[l][(size_t)q] = (uint8_t*)in[l] + (size_t)s->gbase[(size_t)q] * elem;
            rb[l][(size_t)q] = (uint64_t)s->gcnt[(size_t)q] * elem;
        }
        sb[l][(size_t)g->ids[l]] = rb[l][(size_t)g->ids[l]] = 0;
    }
    std::vector<std::vector<uint64_t>> rcnt;
    int rc = tagged_counts(g, XK_DENSE, sb, rcnt, &rb);
    if (rc) return rc;
    return g->take_tr(g->tr->alltoallv(sp, sb, rp, rb));
}

// GRAFT/PRUNE records in ghost receivers' inboxes of plane `parity` go to
// their shards (after the heartbeat: parity 0; after control round r: r+1).
int exchange_control(gsim_group* g, int parity)
{
    const size_t L = g->hs.size();
    const int K = g->K;
    std::vector<std::vector<uint64_t>> scnt(L, std::vector<uint64_t>((size_t)K, 0)), rcnt;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        const size_t TE = (size_t)h->e * (size_t)std::max(1, h->S);
        uint8_t* ctl = extra_ctl(h) + (size_t)parity * TE;
        uint64_t* cany = extra_cany(h) + (size_t)parity * (size_t)h->n;
        if (hipMemsetAsync(s->d_ccnt, 0, sizeof(uint32_t) * K, h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "control count reset");
        const int64_t nghost = s->own_lo + (h->n - s->own_hi);
        PeerRanges pr{};
        pr.K = K;
        for (int q = 0; q <= K; ++q) pr.lo[q] = s->lpeer[(size_t)q];
        hipLaunchKernelGGL(k_ctl_export, dim3(grid_for(nghost)), dim3(256), 0, h->stream, ctl, cany,
                           (const uint32_t*)h->d_row_ptr, (const uint32_t*)s->d_ymap, (const uint64_t*)h->d_smask, pr,
                           h->e, std::max(1, h->t), s->own_lo, s->own_hi, h->n, s->d_cout, s->d_ccnt, s->ccap);
        if (hipMemcpyAsync(s->h_counts, s->d_ccnt, sizeof(uint32_t) * K, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
            hipStreamSynchronize(h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "control counts");
        for (int d = 0; d < K; ++d) {
            if ((int64_t)s->h_counts[d] > s->ccap)
                return g->fail(GSIM_ERANGE, "control exchange queue overflow");
            scnt[l][(size_t)d] = s->h_counts[d];
        }
    }
    int rc = tagged_counts(g, XK_CONTROL, scnt, rcnt);
    if (rc) return rc;
    std::vector<std::vector<const void*>> sp(L, std::vector<const void*>((size_t)K, nullptr));
    std::vector<std::vector<void*>> rp(L, std::vector<void*>((size_t)K, nullptr));
    std::vector<std::vector<uint64_t>> sb(L, std::vector<uint64_t>((size_t)K, 0)), rb = sb;
    std::vector<int64_t> total(L, 0);
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        for (int q = 0; q < K; ++q) total[l] += (int64_t)rcnt[l][(size_t)q];
        (void)hipSetDevice(h->device);
        rc = g->take(h, ensure(h, &s->d_cin, &s->cin_cap, total[l]));
        if (rc) return rc;
        int64_t off = 0;
        for (int q = 0; q < K; ++q) {
            sp[l][(size_t)q] = s->d_cout + (int64_t)q * s->ccap;
            sb[l][(size_t)q] = scnt[l][(size_t)q] * 8;
            rp[l][(size_t)q] = s->d_cin + off;
            rb[l][(size_t)q] = rcnt[l][(size_t)q] * 8;
            off += (int64_t)rcnt[l][(size_t)q];
        }
    }
    rc = g->take_tr(g->tr->alltoallv(sp, sb, rp, rb));
    if (rc) return rc;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        if (!total[l]) continue;
        (void)hipSetDevice(h->device);
        const size_t TE = (size_t)h->e * (size_t)std::max(1, h->S);
        hipLaunchKernelGGL(k_ctl_import, dim3(grid_for(total[l])), dim3(256), 0, h->stream,
                           (const uint64_t*)h->sh->d_cin, total[l], extra_ctl(h) + (size_t)parity * TE,
                           extra_cany(h) + (size_t)parity * (size_t)h->n, (const uint32_t*)h->d_owner,
                           (const uint64_t*)h->d_smask, h->e);
        if (hipGetLastError() != hipSuccess) return g->fail(GSIM_EDEVICE, "k_ctl_import");
    }
    return GSIM_OK;
}

// emitGossip's marks of cross edges into the receiving shards' ghost rows
int exchange_gossip_marks(gsim_group* g)
{
    const size_t L = g->hs.size();
    std::vector<const void*> o1(L), o2(L);
    std::vector<void*> i1(L), i2(L);
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        GossipView gv{};
        if (!deliver_gossip_view(h, &gv)) return GSIM_OK;      // no message state: nothing gossips
        (void)hipSetDevice(h->device);
        const int64_t ncross = s->xoff[(size_t)g->K];
#ifndef GSIM_GSEL_EDGE_ORDER
#define GSIM_GSEL_EDGE_ORDER 1
#endif
        if (ncross && GSIM_GSEL_EDGE_ORDER)
            hipLaunchKernelGGL(k_gsel_export_e, dim3(grid_for(s->own_e_hi - s->own_e_lo)), dim3(256), 0, h->stream,
                               (const uint32_t*)s->d_xpos, s->own_e_lo, s->own_e_hi, (const uint8_t*)gv.gsel,
                               (const uint8_t*)gv.gstate, (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask,
                               h->t, h->e, s->d_gout, s->d_gsout);
        else if (ncross)
            hipLaunchKernelGGL(k_gsel_export, dim3(grid_for(ncross)), dim3(256), 0, h->stream,
                               (const uint32_t*)s->d_xgather, ncross, (const uint8_t*)gv.gsel,
                               (const uint8_t*)gv.gstate, (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask,
                               h->t, h->e, s->d_gout, s->d_gsout);
        o1[l] = s->d_gout; o2[l] = s->d_gsout; i1[l] = s->d_gin; i2[l] = s->d_gsin;
    }
    int rc = exchange_dense(g, o1, i1, 8);
    if (!rc) rc = exchange_dense(g, o2, i2, 1);
    if (rc) return rc;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        GossipView gv{};
        deliver_gossip_view(h, &gv);
        (void)hipSetDevice(h->device);
        const int64_t nghost = s->own_e_lo + (h->e - s->own_e_hi);
        if (nghost)
            hipLaunchKernelGGL(k_gsel_import, dim3(grid_for(nghost)), dim3(256), 0, h->stream,
                               (const uint64_t*)s->d_gin, (const uint8_t*)s->d_gsin, gv.gsel, gv.gstate,
                               (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask, h->t, h->e,
                               s->own_e_lo, s->own_e_hi);
        if (hipGetLastError() != hipSuccess) return g->fail(GSIM_EDEVICE, "k_gsel_import");
    }
    return GSIM_OK;
}

// The router state of cross edges into the ghost rows: what a ghost sender's
// forwarding decision needs (mesh / fanout membership, connected, direct,
// the flood-publish gate on its score of the receiver).
int exchange_router(gsim_group* g)
{
    const size_t L = g->hs.size();
    std::vector<const void*> o1(L), o2(L), o3(L);
    std::vector<void*> i1(L), i2(L), i3(L);
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        const int64_t ncross = s->xoff[(size_t)g->K];
        if (ncross)
            hipLaunchKernelGGL(k_router_export, dim3(grid_for(ncross)), dim3(256), 0, h->stream,
                               (const uint32_t*)s->d_xgather, ncross, (const uint8_t*)h->d_mflags,
                               (const uint8_t*)h->d_rstate, (const uint8_t*)h->d_direct, (const double*)h->d_score,
                               (const uint32_t*)h->d_rev, (const uint32_t*)h->d_owner, (const uint64_t*)h->d_smask,
                               h->th.publish_threshold, h->t, h->e, s->d_rmesh_out,
                               s->d_rfan_out, s->d_rflag_out);
        o1[l] = s->d_rmesh_out; o2[l] = s->d_rfan_out; o3[l] = s->d_rflag_out;
        i1[l] = s->d_rmesh_in; i2[l] = s->d_rfan_in; i3[l] = s->d_rflag_in;
    }
    int rc = exchange_dense(g, o1, i1, 8);
    if (!rc) rc = exchange_dense(g, o2, i2, 8);
    if (!rc) rc = exchange_dense(g, o3, i3, 1);
    if (rc) return rc;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        const int64_t nghost = s->own_e_lo + (h->e - s->own_e_hi);
        GossipView gv{};
        uint64_t* mm = deliver_gossip_view(h, &gv) ? gv.mmask : nullptr;
        const int64_t ngr = s->own_lo + (h->n - s->own_hi);
        if (mm && ngr)
            hipLaunchKernelGGL(k_ghost_mask_clear, dim3(grid_for(ngr * std::max(1, h->t))), dim3(256), 0, h->stream, mm,
                               s->own_lo, s->own_hi, h->n, std::max(1, h->t));
        if (nghost)
            hipLaunchKernelGGL(k_router_import, dim3(grid_for(nghost)), dim3(256), 0, h->stream,
                               (const uint64_t*)s->d_rmesh_in, (const uint64_t*)s->d_rfan_in,
                               (const uint8_t*)s->d_rflag_in, h->d_mflags, h->d_rstate, h->d_direct, s->d_pgate,
                               h->t, h->e, s->own_e_lo, s->own_e_hi, (const uint32_t*)h->d_row_ptr,
                               (const uint32_t*)h->d_owner, h->n, mm, (const uint64_t*)h->d_smask);
        if (hipGetLastError() != hipSuccess) return g->fail(GSIM_EDEVICE, "k_router_import");
        h->score_version++;    // ghost rows' connected / direct bits feed the delivery state
    }
    g->router_dirty = false;
    return GSIM_OK;
}

// The mesh changes control round r made to cross edges (k_handle_control's
// list), to the shards holding their ghost copies.  A list over its capacity
// (seen by every process through the counts) falls back to the full router
// exchange before the next round.
int exchange_router_delta(gsim_group* g)
{
    const size_t L = g->hs.size();
    const int K = g->K;
    constexpr uint64_t kOver = kCountMask;
    std::vector<std::vector<uint64_t>> scnt(L, std::vector<uint64_t>((size_t)K, 0)), rcnt;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        if (hipMemcpyAsync(s->h_counts, s->d_rdel_n, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
            hipStreamSynchronize(h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "router delta count");
        const uint64_t n = s->h_counts[0];
        for (int d = 0; d < K; ++d)
            scnt[l][(size_t)d] = d == g->ids[l] ? 0 : ((int64_t)n > s->rdel_cap ? kOver : n);
    }
    int rc = tagged_counts(g, XK_RDELTA, scnt, rcnt);
    if (rc) return rc;
    bool over = false;
    for (size_t l = 0; l < L; ++l) {
        for (int q = 0; q < K; ++q) over |= rcnt[l][(size_t)q] == kOver || scnt[l][(size_t)q] == kOver;
    }
    std::vector<std::vector<const void*>> sp(L, std::vector<const void*>((size_t)K, nullptr));
    std::vector<std::vector<void*>> rp(L, std::vector<void*>((size_t)K, nullptr));
    std::vector<std::vector<uint64_t>> sb(L, std::vector<uint64_t>((size_t)K, 0)), rb = sb;
    std::vector<int64_t> total(L, 0);
    if (!over) {
        for (size_t l = 0; l < L; ++l) {
            gsim_handle* h = g->hs[l];
            ShardCtx* s = h->sh;
            for (int q = 0; q < K; ++q) total[l] += (int64_t)rcnt[l][(size_t)q];
            (void)hipSetDevice(h->device);
            rc = g->take(h, ensure(h, &s->d_rdel_in, &s->rdel_in_cap, total[l]));
            if (rc) return rc;
            int64_t off = 0;
            for (int q = 0; q < K; ++q) {
                sp[l][(size_t)q] = s->d_rdel;
                sb[l][(size_t)q] = scnt[l][(size_t)q] * 8;
                rp[l][(size_t)q] = s->d_rdel_in + off;
                rb[l][(size_t)q] = rcnt[l][(size_t)q] * 8;
                off += (int64_t)rcnt[l][(size_t)q];
            }
        }
        rc = g->take_tr(g->tr->alltoallv(sp, sb, rp, rb));
        if (rc) return rc;
    }
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        if (!over && total[l]) {
            EdgeBases gb{};
            for (int q = 0; q < K; ++q) gb.b[q] = s->gbase[(size_t)q];
            GossipView gv{};
            uint64_t* mm = deliver_gossip_view(h, &gv) ? gv.mmask : nullptr;
            hipLaunchKernelGGL(k_router_delta, dim3(grid_for(total[l])), dim3(256), 0, h->stream,
                               (const uint64_t*)s->d_rdel_in, total[l], g->ids[l], gb, h->d_mflags,
                               (const uint8_t*)h->d_direct, (const uint32_t*)h->d_row_ptr, (const uint32_t*)h->d_owner,
                               (const uint64_t*)h->d_smask, h->e, h->n, mm);
            if (hipGetLastError() != hipSuccess) return g->fail(GSIM_EDEVICE, "k_router_delta");
        }
        if (hipMemsetAsync(s->d_rdel_n, 0, sizeof(uint32_t), h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "router delta reset");
    }
    if (over) g->router_dirty = true;
    return GSIM_OK;
}

// Round `round`'s forwarders: every shard's owned ones (one list) to every
// shard they have connections into, which imports its ghosts among them.
// Push: only IHAVE reads a ghost's holder round, and the entries carry it, so
// the rounds' exports accumulate and go out once per tick (flush: the round
// whose IHAVE follows), one exchange instead of one per round.
// Push: the tick's holders as bits (deliver_holder_*): every round ORs its
// forwarders into the bits of their first-seen tick; the flush (the first
// round of tick k+1, before its IHAVE) sends tick k's to every shard the
// owned peers have connections into, whose ghosts among them get cells with
// first-seen round kR.  No host synchronisation but the flush's count.
static int exchange_holders(gsim_group* g, int64_t round, bool flush)
{
    const size_t L = g->hs.size();
    const int K = g->K;
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        ProfScope ps(h, GSIM_K_SEND);
        int rc = g->take(h, deliver_holder_accum(h, round));
        if (rc) return rc;
    }
    const int64_t R = g->rounds;
    if (!flush || round < R) return GSIM_OK;
    const int64_t tk = round / R - 1;                      // the tick whose holders go out
    for (gsim_handle* h : g->hs) {
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        ProfScope ps(h, GSIM_K_SEND);
        int rc = g->take(h, deliver_holder_gather(h, (int)(tk & 1)));
        if (!rc && hipMemcpyAsync(s->h_counts, s->d_hn, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream) != hipSuccess)
            rc = g->fail(GSIM_EDEVICE, "holder bits: slot count");
        if (rc) return rc;
    }
    int rc = sync_all(g);
    if (rc) return rc;
    std::vector<std::vector<uint64_t>> scnt(L, std::vector<uint64_t>((size_t)K, 0)), rcnt;
    for (size_t l = 0; l < L; ++l) {
        const ShardCtx* s = g->hs[l]->sh;
        const uint64_t n = s->h_counts[0];
        for (int d = 0; d < K; ++d)
            scnt[l][(size_t)d] = (d == g->ids[l] || !s->xto[(size_t)d] || !n) ? 0 : n * (uint64_t)(1 + s->how);
    }
    rc = tagged_counts(g, XK_FRONTIER, scnt, rcnt);
    if (rc) return rc;
    std::vector<std::vector<const void*>> sp(L, std::vector<const void*>((size_t)K, nullptr));
    std::vector<std::vector<void*>> rp(L, std::vector<void*>((size_t)K, nullptr));
    std::vector<std::vector<uint64_t>> sb(L, std::vector<uint64_t>((size_t)K, 0)), rb = sb;
    std::vector<int64_t> ntask(L, 0);
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        int64_t total = 0;
        for (int q = 0; q < K; ++q) total += (int64_t)rcnt[l][(size_t)q];
        (void)hipSetDevice(h->device);
        rc = g->take(h, ensure(h, &s->d_fin, &s->fin_cap, total));
        if (rc) return rc;
        int64_t off = 0;
        for (int q = 0; q < K; ++q) {
            sp[l][(size_t)q] = s->d_hsend;
            sb[l][(size_t)q] = scnt[l][(size_t)q] * 8;
            rp[l][(size_t)q] = s->d_fin + off;
            rb[l][(size_t)q] = rcnt[l][(size_t)q] * 8;
            // source q's part: its touched slots, then its owned global words each
            const int64_t glo = g->bounds[(size_t)q], ghi = g->bounds[(size_t)q + 1];
            const int64_t nw = ghi > glo ? ((ghi + 63) >> 6) - (glo >> 6) : 0;
            const int64_t c = (int64_t)rcnt[l][(size_t)q];
            HSrc& x = s->h_hsrc[q];
            x.in_off = off;
            x.pbase = (glo >> 6) * 64;
            x.nw = (int32_t)nw;
            x.n = 0;
            if (c) {
                if (nw == 0 || c % (1 + nw))
                    return g->fail(GSIM_ESTATE, "holder bits from shard " + std::to_string(q) + " do not match its range");
                x.n = (int32_t)(c / (1 + nw));
            }
            x.toff = ntask[l];
            ntask[l] += (int64_t)x.n * ((nw + 63) / 64);
            off += c;
        }
    }
    rc = g->take_tr(g->tr->alltoallv(sp, sb, rp, rb));
    if (rc) return rc;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        if (ntask[l] <= 0) continue;
        (void)hipSetDevice(h->device);
        ProfScope ps(h, GSIM_K_SEND);
        if (hipMemcpyAsync(s->d_hsrc, s->h_hsrc, sizeof(HSrc) * (size_t)K, hipMemcpyHostToDevice, h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "holder bits: source table");
        rc = g->take(h, deliver_holder_import(h, round, s->d_fin, s->d_hsrc, K, ntask[l], tk * R));
        if (rc) return rc;
    }
    return GSIM_OK;
}

int exchange_frontier(gsim_group* g, int64_t round, bool flush)
{
    const size_t L = g->hs.size();
    const int K = g->K;
    const bool push = L > 0 && g->hs[0]->sh->push;
    if (push) return exchange_holders(g, round, flush);
    std::vector<std::vector<uint64_t>> scnt(L, std::vector<uint64_t>((size_t)K, 0)), rcnt;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        const int64_t prev = push ? s->fpend : 0;
        for (int attempt = 0; attempt < 2; ++attempt) {
            int rc = g->take(h, deliver_frontier_export(h, round, s->d_fout, s->d_fcnt, s->fcap, push));
            if (rc) return rc;
            if (hipMemcpyAsync(s->h_counts, s->d_fcnt, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
                hipStreamSynchronize(h->stream) != hipSuccess)
                return g->fail(GSIM_EDEVICE, "frontier count");
            const int64_t need = s->h_counts[0];
            if (need <= s->fcap) break;
            if (attempt) return g->fail(GSIM_ERANGE, "frontier export overflow");
            // a busier round (or tick) than any before: grow the list, keep the
            // entries accumulated before this round and export it again (the
            // export only reads the round's state)
            uint64_t* old = s->d_fout;
            s->d_fout = nullptr;
            const int64_t cap = need + need / 2;
            rc = g->take(h, dalloc(h, &s->d_fout, (size_t)cap));
            if (rc) return rc;
            if (prev && stream_copy(h, s->d_fout, old, sizeof(uint64_t) * (size_t)prev, hipMemcpyDeviceToDevice) != hipSuccess)
                return g->fail(GSIM_EDEVICE, "frontier list grow");
            (void)hipFree(old);
            s->fcap = cap;
            const uint32_t pv = (uint32_t)prev;
            if (stream_copy(h, s->d_fcnt, &pv, sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess)
                return g->fail(GSIM_EDEVICE, "frontier count");
        }
        s->fpend = s->h_counts[0];
        for (int d = 0; d < K; ++d)
            scnt[l][(size_t)d] = (d == g->ids[l] || !s->xto[(size_t)d]) ? 0 : (uint64_t)s->fpend;
    }
    if (push && !flush) return GSIM_OK;
    int rc = tagged_counts(g, XK_FRONTIER, scnt, rcnt);
    if (rc) return rc;
    std::vector<std::vector<const void*>> sp(L, std::vector<const void*>((size_t)K, nullptr));
    std::vector<std::vector<void*>> rp(L, std::vector<void*>((size_t)K, nullptr));
    std::vector<std::vector<uint64_t>> sb(L, std::vector<uint64_t>((size_t)K, 0)), rb = sb;
    std::vector<int64_t> total(L, 0);
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        for (int q = 0; q < K; ++q) total[l] += (int64_t)rcnt[l][(size_t)q];
        (void)hipSetDevice(h->device);
        rc = g->take(h, ensure(h, &s->d_fin, &s->fin_cap, total[l]));
        if (rc) return rc;
    }
    for (size_t l = 0; l < L; ++l) {
        ShardCtx* s = g->hs[l]->sh;
        int64_t off = 0;
        for (int q = 0; q < K; ++q) {
            sp[l][(size_t)q] = s->d_fout;
            sb[l][(size_t)q] = scnt[l][(size_t)q] * 8;
            rp[l][(size_t)q] = s->d_fin + off;
            rb[l][(size_t)q] = rcnt[l][(size_t)q] * 8;
            off += (int64_t)rcnt[l][(size_t)q];
        }
    }
    rc = g->take_tr(g->tr->alltoallv(sp, sb, rp, rb));
    if (rc) return rc;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        (void)hipSetDevice(h->device);
        ProfScope ps(h, GSIM_K_SEND);
        rc = g->take(h, deliver_frontier_import(h, round, h->sh->d_fin, total[l]));
        if (rc) return rc;
        if (push) {                                   // the next tick accumulates afresh
            if (hipMemsetAsync(h->sh->d_fcnt, 0, sizeof(uint32_t), h->stream) != hipSuccess)
                return g->fail(GSIM_EDEVICE, "frontier count");
            h->sh->fpend = 0;
        }
    }
    return GSIM_OK;
}

// Copy push: round `round`'s copies from owned senders to
// ghost receivers, bits of (slot, cross edge) set by k_send_tm<PUSH> and
// gathered per destination (the round's active slots, then their segments:
// k_xbits_gather, right after the send), go to the receivers' shards, whose
// k_xbits_deliver applies them (AcceptFrom, the claim of the cell, the
// records) with the round's local copies, before the commit.
int exchange_copies(gsim_group* g, int64_t round)
{
    const size_t L = g->hs.size();
    const int K = g->K;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        if (hipMemcpyAsync(s->h_xcnt, s->d_xn, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "copy bits: slot count");
    }
    int rc = sync_all(g);
    if (rc) return rc;
    std::vector<std::vector<uint64_t>> scnt(L, std::vector<uint64_t>((size_t)K, 0)), rcnt;
    for (size_t l = 0; l < L; ++l) {
        const ShardCtx* s = g->hs[l]->sh;
        const uint64_t n = s->h_xcnt[0];
        for (int d = 0; d < K; ++d) {
            const int64_t xw = s->xwo[(size_t)d + 1] - s->xwo[(size_t)d];
            scnt[l][(size_t)d] = (d == g->ids[l] || xw == 0) ? 0 : n * (uint64_t)(1 + xw);
        }
    }
    rc = tagged_counts(g, XK_COPIES, scnt, rcnt);
    if (rc) return rc;
    std::vector<std::vector<const void*>> sp(L, std::vector<const void*>((size_t)K, nullptr));
    std::vector<std::vector<void*>> rp(L, std::vector<void*>((size_t)K, nullptr));
    std::vector<std::vector<uint64_t>> sb(L, std::vector<uint64_t>((size_t)K, 0)), rb = sb;
    std::vector<int64_t> total(L, 0), ntask(L, 0);
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        for (int q = 0; q < K; ++q) total[l] += (int64_t)rcnt[l][(size_t)q];
        (void)hipSetDevice(h->device);
        rc = g->take(h, ensure(h, &s->d_xrecv, &s->xrecv_cap, total[l]));
        if (rc) return rc;
        int64_t off = 0;
        for (int q = 0; q < K; ++q) {
            sp[l][(size_t)q] = s->d_xsend + (size_t)q * (size_t)s->xsend_cap;
            sb[l][(size_t)q] = scnt[l][(size_t)q] * 8;
            rp[l][(size_t)q] = s->d_xrecv + off;
            rb[l][(size_t)q] = rcnt[l][(size_t)q] * 8;
            // source q's part: its slots' ids, then xw words each (xw from the
            // ghost block of its peers, which is its cross-out list into here)
            const int64_t xw = (s->gcnt[(size_t)q] + 63) / 64;
            const int64_t c = (int64_t)rcnt[l][(size_t)q];
            XSrc& x = s->h_xsrc[q];
            x.in_off = off;
            x.gbase = s->gbase[(size_t)q];
            x.xw = (int32_t)xw;
            x.n = 0;
            if (c) {
                if (xw == 0 || c % (1 + xw)) return g->fail(GSIM_ESTATE, "copy bits from shard " + std::to_string(q) +
                                                                        " do not match its ghost block");
                x.n = (int32_t)(c / (1 + xw));
            }
            x.toff = ntask[l];
            ntask[l] += (int64_t)x.n * ((xw + 63) / 64);
            off += c;
        }
    }
    rc = g->take_tr(g->tr->alltoallv(sp, sb, rp, rb));
    if (rc) return rc;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        if (ntask[l] <= 0) continue;
        (void)hipSetDevice(h->device);
        ProfScope ps(h, GSIM_K_SEND);
        if (hipMemcpyAsync(s->d_xsrc, s->h_xsrc, sizeof(XSrc) * (size_t)K, hipMemcpyHostToDevice, h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "copy bits: source table");
        rc = g->take(h, deliver_xbits_apply(h, round, s->d_xrecv, s->d_xsrc, K, ntask[l]));
        if (rc) return rc;
        g->settle(h);
    }
    return GSIM_OK;
}

// Create the group's shard handles; transport set by the caller.
int group_create(const gsim_peer_score_params* params, const gsim_topic_score_params* topics, int32_t n_topics,
                 const gsim_thresholds* th, const gsim_gossipsub_params* gp, int32_t shards,
                 const std::vector<std::pair<int, int>>& local, gsim_group** out, char* err, size_t errlen)
{
    gsim_group* g = new gsim_group();
    g->K = shards;
    const char* ser = std::getenv("GSIM_GROUP_SERIAL");
    g->serial = ser && ser[0] == '1';
    for (const auto& sd : local) {
        gsim_handle* h = nullptr;
        const int rc = gsim_create(params, topics, n_topics, th, gp, sd.second, &h, err, errlen);
        if (rc) {
            for (gsim_handle* x : g->hs) gsim_destroy(x);
            delete g;
            return rc;
        }
        h->sh = new ShardCtx();
        h->sh->k = sd.first;
        h->sh->K = shards;
        // GSIM_SHARD_PULL=1: the pull exchange (ghost forwarders walked by the
        // receivers' shards; A/B and parity reference for the push)
        const char* pl = std::getenv("GSIM_SHARD_PULL");
        h->sh->push = !(pl && pl[0] == '1');
        g->hs.push_back(h);
        g->ids.push_back(sd.first);
    }
    *out = g;
    return GSIM_OK;
}

}  // namespace

extern "C" {

int gsim_rccl_unique_id(void* out, size_t bytes)
{
    if (!out || bytes < sizeof(ncclUniqueId)) return GSIM_EINVAL;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return GSIM_EDEVICE;
    std::memcpy(out, &id, sizeof(id));
    return GSIM_OK;
}

int gsim_group_create(const gsim_peer_score_params* params, const gsim_topic_score_params* topics, int32_t n_topics,
                      const gsim_thresholds* thresholds, const gsim_gossipsub_params* gossip, int32_t shards,
                      const int32_t* devices, gsim_group** out, char* err, size_t errlen)
{
    if (!out || shards < 1 || shards > GSIM_MAX_SHARDS) return GSIM_EINVAL;
    std::vector<std::pair<int, int>> local;
    for (int s = 0; s < shards; ++s) local.push_back({s, devices ? devices[s] : 0});
    int rc = group_create(params, topics, n_topics, thresholds, gossip, shards, local, out, err, errlen);
    if (rc) return rc;
    auto* t = new LocalTransport();
    t->hs = (*out)->hs;
    (*out)->tr.reset(t);
    return GSIM_OK;
}

int gsim_group_create_rccl(const gsim_peer_score_params* params, const gsim_topic_score_params* topics,
                           int32_t n_topics, const gsim_thresholds* thresholds, const gsim_gossipsub_params* gossip,
                           int32_t shards, int32_t rank, int32_t device, const void* unique_id, gsim_group** out,
                           char* err, size_t errlen)
{
    if (!out || !unique_id || shards < 1 || shards > GSIM_MAX_SHARDS || rank < 0 || rank >= shards) return GSIM_EINVAL;
    int rc = group_create(params, topics, n_topics, thresholds, gossip, shards, {{rank, device}}, out, err, errlen);
    if (rc) return rc;
    auto* t = new RcclTransport();
    t->h = (*out)->hs[0];
    t->k = rank;
    t->K = shards;
    (void)hipSetDevice(device);
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    ncclResult_t nr = ncclCommInitRank(&t->comm, shards, id, rank);
    if (nr != ncclSuccess || hipMalloc((void**)&t->d_cnt, sizeof(uint64_t) * shards * shards) != hipSuccess ||
        hipHostMalloc((void**)&t->h_cnt, sizeof(uint64_t) * shards * shards, 0) != hipSuccess) {
        if (err && errlen)
            std::snprintf(err, errlen, "RCCL communicator: %s", nr != ncclSuccess ? ncclGetErrorString(nr) : "allocation");
        delete t;
        gsim_group_destroy(*out);
        *out = nullptr;
        return GSIM_EDEVICE;
    }
    (*out)->tr.reset(t);
    return GSIM_OK;
}

int gsim_group_create_host(const gsim_peer_score_params* params, const gsim_topic_score_params* topics,
                           int32_t n_topics, const gsim_thresholds* thresholds, const gsim_gossipsub_params* gossip,
                           int32_t shards, int32_t rank, int32_t device, const gsim_host_transport* transport,
                           gsim_group** out, char* err, size_t errlen)
{
    if (!out || !transport || !transport->alltoallv || !transport->allreduce || shards < 1 ||
        shards > GSIM_MAX_SHARDS || rank < 0 || rank >= shards)
        return GSIM_EINVAL;
    int rc = group_create(params, topics, n_topics, thresholds, gossip, shards, {{rank, device}}, out, err, errlen);
    if (rc) return rc;
    auto* t = new HostTransport();
    t->h = (*out)->hs[0];
    t->k = rank;
    t->K = shards;
    t->cb = *transport;
    (*out)->tr.reset(t);
    return GSIM_OK;
}

int gsim_group_destroy(gsim_group* g)
{
    if (!g) return GSIM_OK;
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        (void)hipStreamSynchronize(h->stream);
    }
    g->tr.reset();
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        free_shard_ctx(h);
        gsim_destroy(h);
    }
    delete g;
    return GSIM_OK;
}

const char* gsim_group_last_error(const gsim_group* g) { return g ? g->err.c_str() : "null group"; }

gsim_handle* gsim_group_shard(gsim_group* g, int32_t shard)
{
    if (!g) return nullptr;
    for (size_t l = 0; l < g->hs.size(); ++l)
        if (g->ids[l] == shard) return g->hs[l];
    return nullptr;
}

int gsim_group_bounds(const gsim_group* g, int64_t* bounds)
{
    if (!g || !bounds || g->bounds.empty()) return GSIM_EINVAL;
    std::copy(g->bounds.begin(), g->bounds.end(), bounds);
    return GSIM_OK;
}

int gsim_group_state_written(gsim_group* g)
{
    if (!g) return GSIM_EINVAL;
    g->router_dirty = true;
    return GSIM_OK;
}

int gsim_group_load_graph(gsim_group* g, int64_t n, const uint32_t* row_ptr, const uint32_t* col,
                          const uint8_t* outbound, const uint64_t* subs, const uint32_t* ip_ptr,
                          const uint32_t* ip_ids, uint32_t n_ips, const int64_t* bounds)
{
    if (!g || n <= 0 || !row_ptr || !col) return GSIM_EINVAL;
    const int K = g->K;
    if (K > 1 && n >= 0xFFFFFF) return g->fail(GSIM_ERANGE, "a sharded network holds at most 2^24 - 2 peers");
    g->bounds.assign((size_t)K + 1, 0);
    if (bounds) {
        std::copy(bounds, bounds + K + 1, g->bounds.begin());
    } else {
        const int rc = gsim_shard_partition(n, row_ptr, subs, K, g->bounds.data());
        if (rc) return g->fail(rc, "cannot partition the network into " + std::to_string(K) + " shards");
    }
    g->N = n;
    g->E = row_ptr[n];
    g->gid.assign(g->hs.size(), {});
    g->gidx.assign(g->hs.size(), {});
    g->sub.assign(subs ? subs : nullptr, subs ? subs + n : nullptr);
    g->row_ptr.assign(row_ptr, row_ptr + n + 1);
    g->msgs = false;
    g->router_dirty = true;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        gsim_handle* h = g->hs[l];
        ShardLayout L;
        std::string e;
        int rc = build_layout(n, row_ptr, col, g->bounds.data(), K, g->ids[l], &L, &e);
        if (rc) return g->fail(rc, e);
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        (void)hipStreamSynchronize(h->stream);
        free_shard_bufs(s);
        s->own_lo = L.own_lo; s->own_hi = L.own_hi; s->own_e_lo = L.own_e_lo; s->own_e_hi = L.own_e_hi;
        s->N_global = n; s->E_global = g->E;
        s->geid_base = L.own_e_hi > L.own_e_lo ? (int64_t)L.gidx[(size_t)L.own_e_lo] : 0;
        s->bounds = g->bounds; s->lpeer = L.lpeer; s->gbase = L.gbase; s->gcnt = L.gcnt;
        s->xoff.assign((size_t)K + 1, 0);
        for (int q = 0; q < K; ++q) s->xoff[(size_t)q + 1] = s->xoff[(size_t)q] + (int64_t)L.crossout[(size_t)q].size();
        // the local inputs
        std::vector<uint8_t> ob((size_t)L.e_loc, 0);
        if (outbound) for (int64_t x = 0; x < L.e_loc; ++x) ob[(size_t)x] = outbound[L.gidx[(size_t)x]];
        std::vector<uint64_t> sb((size_t)L.n_loc, 0);
        if (subs) for (int64_t x = 0; x < L.n_loc; ++x) sb[(size_t)x] = subs[L.gid[(size_t)x]];
        std::vector<uint32_t> ipp, ipi;
        if (ip_ptr) {
            ipp.assign((size_t)L.n_loc + 1, 0);
            for (int64_t x = 0; x < L.n_loc; ++x) {
                const uint32_t gg = L.gid[(size_t)x];
                for (uint32_t q = ip_ptr[gg]; q < ip_ptr[gg + 1]; ++q) ipi.push_back(ip_ids[q]);
                ipp[(size_t)x + 1] = (uint32_t)ipi.size();
            }
        }
        (void)hipSetDevice(h->device);
        rc = gsim_load_graph(h, L.n_loc, L.row_ptr.data(), L.col.data(), ob.data(), subs ? sb.data() : nullptr,
                             ip_ptr ? ipp.data() : nullptr, ip_ptr ? ipi.data() : nullptr, n_ips);
        if (rc) return g->take(h, rc);
        // device bookkeeping
        std::vector<uint32_t> xg;
        xg.reserve((size_t)L.n_cross);
        for (int q = 0; q < K; ++q) xg.insert(xg.end(), L.crossout[(size_t)q].begin(), L.crossout[(size_t)q].end());
        std::vector<uint32_t> xpos((size_t)L.e_loc, 0xFFFFFFFFu);
        for (size_t q = 0; q < xg.size(); ++q) xpos[xg[q]] = (uint32_t)q;
        std::vector<uint32_t> g2l((size_t)n, kNone);
        for (int64_t x = 0; x < L.n_loc; ++x) g2l[L.gid[(size_t)x]] = (uint32_t)x;
        // the edges of each row into owned peers, in row order: the copies
        // this shard delivers (ghost rows: all of them)
        std::vector<uint32_t> sptr((size_t)L.n_loc + 1, 0), sedge;
        sedge.reserve((size_t)L.e_loc);
        for (int64_t x = 0; x < L.n_loc; ++x) {
            for (uint32_t q = L.row_ptr[(size_t)x]; q < L.row_ptr[(size_t)x + 1]; ++q)
                if ((int64_t)L.col[q] >= L.own_lo && (int64_t)L.col[q] < L.own_hi) sedge.push_back(q);
            sptr[(size_t)x + 1] = (uint32_t)sedge.size();
            s->send_max = std::max<int64_t>(s->send_max, sptr[(size_t)x + 1] - sptr[(size_t)x]);
        }
        s->send_edges = (int64_t)sedge.size();
        s->xto.assign((size_t)K, 0);
        for (int q = 0; q < K; ++q) s->xto[(size_t)q] = L.crossout[(size_t)q].empty() ? 0 : 1;
        const int64_t ncross = L.n_cross;
        if ((rc = dalloc(h, &s->d_gid, (size_t)L.n_loc)) || (rc = dalloc(h, &s->d_g2l, (size_t)n)) ||
            (rc = dalloc(h, &s->d_sptr, sptr.size())) || (rc = dalloc(h, &s->d_xq, (size_t)L.e_loc)) ||
            (rc = dalloc(h, &s->d_sedge, sedge.size())) ||
            (rc = dalloc(h, &s->d_ymap, (size_t)L.e_loc)) || (rc = dalloc(h, &s->d_xgather, xg.size())) ||
            (rc = dalloc(h, &s->d_xpos, (size_t)L.e_loc)) ||
            (rc = dalloc(h, &s->d_pgate, (size_t)L.e_loc)) ||
            (rc = dalloc(h, &s->d_rmesh_out, (size_t)ncross)) || (rc = dalloc(h, &s->d_rfan_out, (size_t)ncross)) ||
            (rc = dalloc(h, &s->d_rflag_out, (size_t)ncross)) || (rc = dalloc(h, &s->d_rmesh_in, (size_t)L.e_loc)) ||
            (rc = dalloc(h, &s->d_rfan_in, (size_t)L.e_loc)) || (rc = dalloc(h, &s->d_rflag_in, (size_t)L.e_loc)))
            return g->take(h, rc);
        if (!s->h_counts && hipHostMalloc((void**)&s->h_counts, sizeof(uint32_t) * GSIM_MAX_SHARDS, 0) != hipSuccess)
            return g->fail(GSIM_ENOMEM, "pinned scratch");
        hipError_t he = stream_copy(h, s->d_gid, L.gid.data(), L.gid.size() * 4, hipMemcpyHostToDevice);
        if (he == hipSuccess) he = stream_copy(h, s->d_g2l, g2l.data(), g2l.size() * 4, hipMemcpyHostToDevice);
        if (he == hipSuccess) he = stream_copy(h, s->d_sptr, sptr.data(), sptr.size() * 4, hipMemcpyHostToDevice);
        if (he == hipSuccess) he = stream_copy(h, s->d_xq, L.xq.data(), L.xq.size() * 4, hipMemcpyHostToDevice);
        if (he == hipSuccess && !sedge.empty())
            he = stream_copy(h, s->d_sedge, sedge.data(), sedge.size() * 4, hipMemcpyHostToDevice);
        if (he == hipSuccess && !xg.empty()) he = stream_copy(h, s->d_xgather, xg.data(), xg.size() * 4, hipMemcpyHostToDevice);
        if (he == hipSuccess) he = stream_copy(h, s->d_xpos, xpos.data(), xpos.size() * 4, hipMemcpyHostToDevice);
        if (he == hipSuccess) he = stream_fill(h, s->d_ymap, 0xFF, (size_t)L.e_loc * 4);
        if (he == hipSuccess) he = stream_fill(h, s->d_pgate, 0, (size_t)L.e_loc);
        if (he != hipSuccess) return g->fail(GSIM_EDEVICE, "shard tables upload");
        // copy push: each local peer's shard; the cross edges' indices at the
        // receivers' shards follow once every shard's ghost blocks are known
        std::vector<uint8_t> psh((size_t)L.n_loc, 0);
        for (int q = 0; q < K; ++q)
            for (int64_t x = L.lpeer[(size_t)q]; x < L.lpeer[(size_t)q + 1]; ++x) psh[(size_t)x] = (uint8_t)q;
        if ((rc = dalloc(h, &s->d_pshard, psh.size())) || (rc = dalloc(h, &s->d_xre, (size_t)L.e_loc)))
            return g->take(h, rc);
        if (stream_copy(h, s->d_pshard, psh.data(), psh.size(), hipMemcpyHostToDevice) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "shard tables upload");
        // copy bits: per destination a word-aligned segment of a slot's row, a
        // cross edge's bit at its position in the cross-out list
        s->xwo.assign((size_t)K + 1, 0);
        for (int q = 0; q < K; ++q)
            s->xwo[(size_t)q + 1] = s->xwo[(size_t)q] + ((int64_t)L.crossout[(size_t)q].size() + 63) / 64;
        s->xbw = s->xwo[(size_t)K];
        if (s->xbw * 64 >= (int64_t)0xFFFFFFFFll) return g->fail(GSIM_ERANGE, "too many cross edges for the copy bits");
        {
            std::vector<uint32_t> xwq((size_t)L.e_loc, 0xFFFFFFFFu);
            for (int q = 0; q < K; ++q)
                for (size_t x = 0; x < L.crossout[(size_t)q].size(); ++x)
                    xwq[L.crossout[(size_t)q][x]] = (uint32_t)(s->xwo[(size_t)q] * 64 + (int64_t)x);
            if ((rc = dalloc(h, &s->d_xwq, xwq.size())) || (rc = dalloc(h, &s->d_xwo, s->xwo.size())))
                return g->take(h, rc);
            if (stream_copy(h, s->d_xwq, xwq.data(), xwq.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
                stream_copy(h, s->d_xwo, s->xwo.data(), s->xwo.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
                return g->fail(GSIM_EDEVICE, "shard tables upload");
        }
        g->gid[l] = L.gid;
        g->gidx[l] = L.gidx;
    }
    // control destinations: a ghost-row edge's owned-row edge in the ghost's
    // shard = that shard's cross-out list into this one (ymap, ghost blocks)
    std::vector<const void*> xo(g->hs.size());
    std::vector<void*> ym(g->hs.size());
    for (size_t l = 0; l < g->hs.size(); ++l) {
        xo[l] = g->hs[l]->sh->d_xgather;
        ym[l] = g->hs[l]->sh->d_ymap;
    }
    int rc = exchange_dense(g, xo, ym, 4);
    if (rc) return rc;
    // copy push: shard d's ghost block of this shard's peers starts at its
    // local edge gbase_d[this] (one count exchange)
    {
        const size_t Ls = g->hs.size();
        std::vector<std::vector<uint64_t>> sc(Ls, std::vector<uint64_t>((size_t)K, 0)), rcv;
        for (size_t l = 0; l < Ls; ++l)
            for (int q = 0; q < K; ++q) sc[l][(size_t)q] = (uint64_t)g->hs[l]->sh->gbase[(size_t)q];
        rc = tagged_counts(g, XK_GBASE, sc, rcv);
        if (rc) return rc;
        for (size_t l = 0; l < Ls; ++l) {
            gsim_handle* h = g->hs[l];
            ShardCtx* s = h->sh;
            s->rbase.assign((size_t)K, 0);
            EdgeBases rb{};
            for (int q = 0; q < K; ++q) rb.b[q] = s->rbase[(size_t)q] = (int64_t)rcv[l][(size_t)q];
            (void)hipSetDevice(h->device);
            hipLaunchKernelGGL(k_xre_build, dim3(grid_for(h->e)), dim3(256), 0, h->stream, (const uint32_t*)s->d_xq,
                               (const uint32_t*)h->d_col, (const uint8_t*)s->d_pshard, rb, s->d_xre, h->e);
            if (hipGetLastError() != hipSuccess) return g->fail(GSIM_EDEVICE, "k_xre_build");
        }
    }
    // peer exchange: PX lists to ghosts (k_px_emit's remote path), per destination
    for (gsim_handle* h : g->hs) {
        ShardCtx* s = h->sh;
        if (!px_enabled(h)) continue;
        (void)hipSetDevice(h->device);
        // a tick's PX lists to one shard: PrunePeers entries per cross edge into it,
        // four PX PRUNEs per cross edge and tick (the heartbeat's and the two
        // control rounds' GRAFT replies, of several topics: c5's hubs overflowed
        // one; an overflow fails gsim_group_px_connect)
        int64_t xmax = 0;
        for (int q = 0; q < K; ++q) xmax = std::max<int64_t>(xmax, s->xoff[(size_t)q + 1] - s->xoff[(size_t)q]);
        s->pxcap = std::max<int64_t>(1 << 16, 4 * (int64_t)std::max(1, h->gp.prune_peers) * xmax);
        if ((rc = dalloc(h, &s->d_pxout, (size_t)(K * s->pxcap))) || (rc = dalloc(h, &s->d_pxcnt, (size_t)K + 1)))
            return g->take(h, rc);
        if (stream_fill(h, s->d_pxcnt, 0, sizeof(uint32_t) * ((size_t)K + 1)) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "PX list counts");
    }
    return sync_all(g);
}

int gsim_group_msgs_init(gsim_group* g, const gsim_msg_config* cfg)
{
    if (!g || !cfg) return GSIM_EINVAL;
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        int rc = gsim_msgs_init(h, cfg);
        if (rc) return g->take(h, rc);
        ShardCtx* s = h->sh;
        const int K = g->K;
        int64_t gmax = 0;
        for (int q = 0; q < K; ++q) gmax = std::max<int64_t>(gmax, s->gcnt[(size_t)q]);
        // a round's forwarders per destination shard: each owned peer once per
        // message it first saw in the round before (grown on demand);
        // max_frontier sets the initial size
        s->fcap = cfg->max_frontier > 0 ? cfg->max_frontier : std::max<int64_t>(8 * (s->own_hi - s->own_lo), 1 << 16);
        s->ccap = std::max<int64_t>(4 * gmax, 1 << 14);
        const int64_t ncross = s->xoff[(size_t)K];
        rc = GSIM_OK;
        auto A = [&](auto** p, size_t n) { if (!rc) rc = dalloc(h, p, n); };
        if (!s->d_rdel) {
            s->rdel_cap = std::max<int64_t>(1 << 16, (s->own_e_hi - s->own_e_lo) / 16);
            A(&s->d_rdel, (size_t)s->rdel_cap);
            A(&s->d_rdel_n, 1);
            if (!rc && stream_fill(h, s->d_rdel_n, 0, 4) != hipSuccess) return g->fail(GSIM_EDEVICE, "router delta count");
        }
        if (s->d_fout) { (void)hipFree(s->d_fout); s->d_fout = nullptr; }
        A(&s->d_fout, (size_t)s->fcap);
        if (!s->d_fcnt) A(&s->d_fcnt, 1);
        if (!rc && stream_fill(h, s->d_fcnt, 0, sizeof(uint32_t)) != hipSuccess) return g->fail(GSIM_EDEVICE, "frontier count");
        s->fpend = 0;
        if (!s->d_cout) {
            A(&s->d_cout, (size_t)(K * s->ccap));
            A(&s->d_ccnt, (size_t)K);
            A(&s->d_gout, (size_t)ncross);
            A(&s->d_gsout, (size_t)ncross);
            A(&s->d_gin, (size_t)h->e);
            A(&s->d_gsin, (size_t)h->e);
        }
        if (!rc && s->push && s->hring != cfg->ring) {
            // a tick's holders as bits over the owned peers' global words
            for (auto* p : {(void*)s->d_hbits, (void*)s->d_hsend}) if (p) (void)hipFree(p);
            s->d_hbits = nullptr; s->d_hsend = nullptr;
            const int64_t glo = s->bounds[(size_t)s->k], ghi = s->bounds[(size_t)s->k + 1];
            s->how = ghi > glo ? ((ghi + 63) >> 6) - (glo >> 6) : 0;
            const size_t hw = (size_t)(cfg->ring + 31) / 32;
            A(&s->d_hbits, (size_t)(2 * (int64_t)cfg->ring * s->how));
            A(&s->d_hsend, (size_t)((int64_t)cfg->ring * (1 + s->how)));
            if (!s->d_hslots) A(&s->d_hslots, 2 * hw);
            if (!s->d_hn) A(&s->d_hn, 1);
            if (!s->d_hsrc) A(&s->d_hsrc, (size_t)K);
            if (!rc && !s->h_hsrc && hipHostMalloc((void**)&s->h_hsrc, sizeof(HSrc) * (size_t)K, 0) != hipSuccess)
                return g->fail(GSIM_ENOMEM, "pinned scratch");
            if (!rc && (stream_fill(h, s->d_hbits, 0, sizeof(uint64_t) * (size_t)(2 * (int64_t)cfg->ring * s->how)) != hipSuccess ||
                        stream_fill(h, s->d_hslots, 0, sizeof(uint32_t) * 2 * hw) != hipSuccess))
                return g->fail(GSIM_EDEVICE, "holder bits");
            if (!rc) s->hring = cfg->ring;
        } else if (!rc && s->push) {   // a new message configuration: no holders pending
            const size_t hw = (size_t)(cfg->ring + 31) / 32;
            if (stream_fill(h, s->d_hbits, 0, sizeof(uint64_t) * (size_t)(2 * (int64_t)cfg->ring * s->how)) != hipSuccess ||
                stream_fill(h, s->d_hslots, 0, sizeof(uint32_t) * 2 * hw) != hipSuccess)
                return g->fail(GSIM_EDEVICE, "holder bits");
        }
        if (!rc && s->push && s->xring != cfg->ring) {
            // a round's copies to ghost receivers: a bit per (slot, cross edge);
            // per destination the active slots' ids and segments go out
            if (s->d_xbits) { (void)hipFree(s->d_xbits); s->d_xbits = nullptr; }
            if (s->d_xsend) { (void)hipFree(s->d_xsend); s->d_xsend = nullptr; }
            int64_t xwmax = 0;
            for (int q = 0; q < K; ++q) xwmax = std::max<int64_t>(xwmax, s->xwo[(size_t)q + 1] - s->xwo[(size_t)q]);
            s->xsend_cap = (int64_t)cfg->ring * (1 + xwmax);
            A(&s->d_xbits, (size_t)((int64_t)cfg->ring * s->xbw));
            A(&s->d_xsend, (size_t)(K * s->xsend_cap));
            if (!s->d_xn) A(&s->d_xn, 1);
            if (!s->d_xsrc) A(&s->d_xsrc, (size_t)K);
            if (!rc && !s->h_xcnt && hipHostMalloc((void**)&s->h_xcnt, sizeof(uint32_t) * 2, 0) != hipSuccess)
                return g->fail(GSIM_ENOMEM, "pinned scratch");
            if (!rc && !s->h_xsrc && hipHostMalloc((void**)&s->h_xsrc, sizeof(XSrc) * (size_t)K, 0) != hipSuccess)
                return g->fail(GSIM_ENOMEM, "pinned scratch");
            if (!rc && stream_fill(h, s->d_xbits, 0, sizeof(uint64_t) * (size_t)((int64_t)cfg->ring * s->xbw)) != hipSuccess)
                return g->fail(GSIM_EDEVICE, "copy bits");
            if (!rc) s->xring = cfg->ring;
        }
        if (rc) return g->take(h, rc);
        if (stream_fill(h, s->d_gin, 0, (size_t)h->e * 8) != hipSuccess || stream_fill(h, s->d_gsin, 0, (size_t)h->e) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "gossip mark buffers");
    }
    g->ring = cfg->ring;
    g->rounds = cfg->rounds;
    g->msgs = true;
    return sync_all(g);
}

#define GROUP_EACH(g, call)                                      \
    do {                                                         \
        if (!(g)) return GSIM_EINVAL;                            \
        for (gsim_handle* h : (g)->hs) {                         \
            int rc_ = (call);                                    \
            if (rc_) return (g)->take(h, rc_);                   \
            (g)->settle(h);                                      \
        }                                                        \
    } while (0)

int gsim_group_set_seed(gsim_group* g, uint64_t seed) { GROUP_EACH(g, gsim_set_seed(h, seed)); return GSIM_OK; }

int gsim_group_fill_synthetic(gsim_group* g, uint64_t seed, int64_t now, double p_mesh)
{
    GROUP_EACH(g, gsim_fill_synthetic(h, seed, now, p_mesh));
    g->router_dirty = true;
    return GSIM_OK;
}

int gsim_group_set_app_score(gsim_group* g, const double* p5)
{
    if (!g || !p5) return GSIM_EINVAL;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        std::vector<double> v(g->gid[l].size());
        for (size_t x = 0; x < v.size(); ++x) v[x] = p5[g->gid[l][x]];
        const int rc = gsim_set_app_score(g->hs[l], v.data());
        if (rc) return g->take(g->hs[l], rc);
    }
    return GSIM_OK;
}

int gsim_group_set_ip_whitelist(gsim_group* g, const uint8_t* white)
{
    GROUP_EACH(g, gsim_set_ip_whitelist(h, white));
    return GSIM_OK;
}

int gsim_group_set_ips(gsim_group* g, const uint32_t* ip_ptr, const uint32_t* ip_ids, uint32_t n_ips)
{
    if (!g || !ip_ptr) return GSIM_EINVAL;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        std::vector<uint32_t> ipp(g->gid[l].size() + 1, 0), ipi;
        for (size_t x = 0; x < g->gid[l].size(); ++x) {
            const uint32_t gg = g->gid[l][x];
            for (uint32_t q = ip_ptr[gg]; q < ip_ptr[gg + 1]; ++q) ipi.push_back(ip_ids[q]);
            ipp[x + 1] = (uint32_t)ipi.size();
        }
        const int rc = gsim_set_ips(g->hs[l], ipp.data(), ipi.data(), n_ips);
        if (rc) return g->take(g->hs[l], rc);
    }
    return GSIM_OK;
}

int gsim_group_set_direct_peers(gsim_group* g, const uint8_t* flags)
{
    if (!g) return GSIM_EINVAL;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        int rc;
        if (!flags) {
            rc = gsim_set_direct_peers(g->hs[l], nullptr);
        } else {
            std::vector<uint8_t> v(g->gidx[l].size());
            for (size_t x = 0; x < v.size(); ++x) v[x] = flags[g->gidx[l][x]];
            rc = gsim_set_direct_peers(g->hs[l], v.data());
        }
        if (rc) return g->take(g->hs[l], rc);
    }
    g->router_dirty = true;
    return GSIM_OK;
}

int gsim_group_set_peer_behaviour(gsim_group* g, const uint8_t* flags)
{
    if (!g || !flags) return GSIM_EINVAL;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        std::vector<uint8_t> v(g->gid[l].size());
        for (size_t x = 0; x < v.size(); ++x) v[x] = flags[g->gid[l][x]];
        const int rc = gsim_set_peer_behaviour(g->hs[l], v.data());
        if (rc) return g->take(g->hs[l], rc);
    }
    return GSIM_OK;
}

int gsim_group_set_topic_params(gsim_group* g, int32_t topic, const gsim_topic_score_params* p)
{
    GROUP_EACH(g, gsim_set_topic_params(h, topic, p));
    return GSIM_OK;
}

int gsim_group_refresh_scores(gsim_group* g, int64_t now)
{
    GROUP_EACH(g, gsim_refresh_scores(h, now));
    g->router_dirty = true;                          // the flood-publish gate reads the new snapshot
    return GSIM_OK;
}

int gsim_group_heartbeat(gsim_group* g, uint64_t tick, int64_t now)
{
    GROUP_EACH(g, gsim_heartbeat(h, tick, now));
    g->router_dirty = true;                          // meshes and fanouts changed
    int rc = exchange_control(g, 0);                 // GRAFT/PRUNE for control round 0
    if (!rc) rc = exchange_gossip_marks(g);
    return rc;
}

int gsim_group_publish(gsim_group* g, const gsim_msg* msgs, int32_t count, int64_t round)
{
    if (!g || count < 0 || (count > 0 && !msgs)) return GSIM_EINVAL;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        std::vector<gsim_msg> v(msgs, msgs + count);
        const std::vector<uint32_t>& gid = g->gid[l];
        for (auto& m : v) {
            auto it = std::lower_bound(gid.begin(), gid.end(), m.origin);
            m.origin = (it != gid.end() && *it == m.origin) ? (uint32_t)(it - gid.begin()) : kNone;
        }
        const int rc = gsim_publish(g->hs[l], v.data(), count, round);
        if (rc) return g->take(g->hs[l], rc);
    }
    // an origin outside its topic may have chosen new fanout peers
    for (int32_t q = 0; q < count; ++q)
        if (g->sub.empty() || !((g->sub[msgs[q].origin] >> msgs[q].topic) & 1ull)) g->router_dirty = true;
    return GSIM_OK;
}

int gsim_group_round(gsim_group* g, int64_t round)
{
    if (!g) return GSIM_EINVAL;
    if (!g->msgs) return g->fail(GSIM_ESTATE, "gsim_group_msgs_init not called");
    int rc = GSIM_OK;
    const bool push = g->hs.empty() || g->hs[0]->sh->push;
    // pull: the ghosts' forwarding state of this round (push: the senders'
    // shards decide, nothing reads a ghost row's router state)
    if (g->router_dirty && !push) {
        rc = exchange_router(g);
        if (rc) return rc;
    }
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        rc = deliver_round_prepare(h, round);        // commits of the last round: fresh forwarders
        if (rc) return g->take(h, rc);
        g->settle(h);
    }
    rc = exchange_frontier(g, round, round % g->rounds == 0);   // the ghosts among them (push: once per tick)
    if (rc) return rc;
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        rc = deliver_round_send(h, round);
        if (rc) return g->take(h, rc);
        g->settle(h);
    }
    if (push) {
        rc = exchange_copies(g, round);              // copies to other shards' peers
        if (rc) return rc;
    }
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        rc = deliver_round_post(h, round);
        if (!rc) rc = deliver_round_control(h, round);
        if (rc) return g->take(h, rc);
        g->settle(h);
    }
    const int64_t r = round % g->rounds;
    if (r < 2) {
        rc = exchange_control(g, (int)((r + 1) & 1));   // PRUNE replies for the next control round
        if (!rc && !push) rc = exchange_router_delta(g);   // the meshes control changed, on cross edges
        if (rc) return rc;
    }
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        rc = deliver_round_ihave(h, round);             // ghost advertisers: their cells
        if (!rc) rc = deliver_round_validate(h, round);  // validations completing (gsim_msg.vdelay)
        if (rc) return g->take(h, rc);
        g->settle(h);
        deliver_round_end(h, round);
    }
    return GSIM_OK;
}

int gsim_group_set_connections(gsim_group* g, const uint32_t* pairs, int32_t count, int32_t up, int64_t now)
{
    if (!g || count < 0 || (count > 0 && !pairs)) return GSIM_EINVAL;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        const std::vector<uint32_t>& gid = g->gid[l];
        ShardCtx* s = g->hs[l]->sh;
        auto loc = [&](uint32_t p) -> int64_t {
            auto it = std::lower_bound(gid.begin(), gid.end(), p);
            return (it != gid.end() && *it == p) ? (int64_t)(it - gid.begin()) : -1;
        };
        std::vector<uint32_t> v;
        for (int32_t q = 0; q < count; ++q) {
            const int64_t a = loc(pairs[2 * q]), b = loc(pairs[2 * q + 1]);
            const bool own_a = a >= s->own_lo && a < s->own_hi, own_b = b >= s->own_lo && b < s->own_hi;
            if (!own_a && !own_b) continue;                  // both endpoints elsewhere
            if (a < 0 || b < 0) return g->fail(GSIM_EINVAL, "pair " + std::to_string(q) + " is not a connection");
            v.push_back((uint32_t)a);
            v.push_back((uint32_t)b);
        }
        const int rc = gsim_set_connections(g->hs[l], v.data(), (int32_t)(v.size() / 2), up, now);
        if (rc) return g->take(g->hs[l], rc);
    }
    g->router_dirty = true;
    return GSIM_OK;
}

// The connector (gossipsub.go:941-973) over the shards, run between ticks by
// every rank: (1) the PX lists PRUNEs carried to other shards' peers are
// delivered and checked there (handlePrune's acceptPXThreshold, a known
// address, not connected: k_px_import); (2) every shard's attempts (asker,
// peer) go to every rank, which resolves each pair once as gsim_px_connect
// does — the asker dials, the lower id when both asked; (3) gs.outbound is set
// on the owned ends and the connections are made with AddPeer at both ends
// (gsim_group_set_connections).
int gsim_group_px_connect(gsim_group* g, int64_t now, uint32_t* pairs, int64_t cap, int64_t* n_connected)
{
    if (!g || !n_connected) return GSIM_EINVAL;
    *n_connected = 0;
    const size_t L = g->hs.size();
    const int K = g->K;
    if (L == 0 || !px_enabled(g->hs[0])) return GSIM_OK;      // WithPeerExchange is off
    // (1) PX lists to the pruned peers' shards
    std::vector<std::vector<uint64_t>> scnt(L, std::vector<uint64_t>((size_t)K, 0)), rcnt;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        if (hipMemcpyAsync(s->h_counts, s->d_pxcnt, sizeof(uint32_t) * ((size_t)K + 1), hipMemcpyDeviceToHost,
                           h->stream) != hipSuccess || hipStreamSynchronize(h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "PX list counts");
        if (s->h_counts[K]) return g->fail(GSIM_ERANGE, "PX list overflow");
        for (int d = 0; d < K; ++d) scnt[l][(size_t)d] = d == g->ids[l] ? 0 : s->h_counts[d];
    }
    int rc = tagged_counts(g, XK_PX, scnt, rcnt);
    if (rc) return rc;
    std::vector<std::vector<const void*>> sp(L, std::vector<const void*>((size_t)K, nullptr));
    std::vector<std::vector<void*>> rp(L, std::vector<void*>((size_t)K, nullptr));
    std::vector<std::vector<uint64_t>> sb(L, std::vector<uint64_t>((size_t)K, 0)), rb = sb;
    std::vector<int64_t> total(L, 0);
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        for (int q = 0; q < K; ++q) total[l] += (int64_t)rcnt[l][(size_t)q];
        (void)hipSetDevice(h->device);
        rc = g->take(h, ensure(h, &s->d_pxin, &s->pxin_cap, std::max<int64_t>(total[l], 1)));
        if (rc) return rc;
        int64_t off = 0;
        for (int q = 0; q < K; ++q) {
            sp[l][(size_t)q] = s->d_pxout + (size_t)q * (size_t)s->pxcap;
            sb[l][(size_t)q] = scnt[l][(size_t)q] * 8;
            rp[l][(size_t)q] = s->d_pxin + off;
            rb[l][(size_t)q] = rcnt[l][(size_t)q] * 8;
            off += (int64_t)rcnt[l][(size_t)q];
        }
    }
    rc = g->take_tr(g->tr->alltoallv(sp, sb, rp, rb));
    if (rc) return rc;
    // (2) every shard's attempts, to every rank
    std::vector<std::vector<uint64_t>> acnt(L, std::vector<uint64_t>((size_t)K, 0));
    std::vector<std::vector<uint64_t>> own(L);
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        rc = g->take(h, px_import(h, s->d_pxin, total[l]));
        if (!rc) rc = g->take(h, px_leave_import(h, (const uint32_t*)s->d_g2l));   // Leave's, to owned peers
        if (!rc) rc = g->take(h, px_asks(h, s->d_pxout, s->d_pxcnt, (int64_t)K * s->pxcap));
        if (rc) return rc;
        if (hipMemcpyAsync(s->h_counts, s->d_pxcnt, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
            hipStreamSynchronize(h->stream) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "PX attempts count");
        const int64_t na = s->h_counts[0];
        if (na > (int64_t)K * s->pxcap) return g->fail(GSIM_ERANGE, "PX attempts overflow");
        own[l].resize((size_t)na);
        if (na && stream_copy(h, own[l].data(), s->d_pxout, sizeof(uint64_t) * (size_t)na, hipMemcpyDeviceToHost) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "PX attempts readback");
        if (stream_fill(h, s->d_pxcnt, 0, sizeof(uint32_t) * ((size_t)K + 1)) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "PX list counts");
        for (int d = 0; d < K; ++d) acnt[l][(size_t)d] = d == g->ids[l] ? 0 : (uint64_t)na;
    }
    rc = tagged_counts(g, XK_PXA, acnt, rcnt);
    if (rc) return rc;
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        total[l] = 0;
        for (int q = 0; q < K; ++q) total[l] += (int64_t)rcnt[l][(size_t)q];
        (void)hipSetDevice(h->device);
        rc = g->take(h, ensure(h, &s->d_pxin, &s->pxin_cap, std::max<int64_t>(total[l], 1)));
        if (rc) return rc;
        int64_t off = 0;
        for (int q = 0; q < K; ++q) {
            sp[l][(size_t)q] = s->d_pxout;
            sb[l][(size_t)q] = acnt[l][(size_t)q] * 8;
            rp[l][(size_t)q] = s->d_pxin + off;
            rb[l][(size_t)q] = rcnt[l][(size_t)q] * 8;
            off += (int64_t)rcnt[l][(size_t)q];
        }
    }
    rc = g->take_tr(g->tr->alltoallv(sp, sb, rp, rb));
    if (rc) return rc;
    // every attempt of the job (this process's shards' own, the others' received)
    std::vector<uint64_t> asks;
    for (size_t l = 0; l < L; ++l) asks.insert(asks.end(), own[l].begin(), own[l].end());
    if (L < (size_t)K) {        // one shard per process: the other ranks' lists (in-process: all are local)
        gsim_handle* h = g->hs[0];
        std::vector<uint64_t> in((size_t)total[0]);
        (void)hipSetDevice(h->device);
        if (total[0] && stream_copy(h, in.data(), h->sh->d_pxin, sizeof(uint64_t) * in.size(), hipMemcpyDeviceToHost) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "PX attempts readback");
        asks.insert(asks.end(), in.begin(), in.end());
    }
    // resolve: per unordered pair, the asker dials (the lower id when both asked)
    std::vector<std::pair<uint64_t, uint32_t>> keyed;     // (lo | hi << 32, bit 1: lo asked, bit 2: hi asked)
    keyed.reserve(asks.size());
    for (uint64_t v : asks) {
        const uint32_t a_ = (uint32_t)v, b_ = (uint32_t)(v >> 32);
        const uint32_t lo = std::min(a_, b_), hi = std::max(a_, b_);
        keyed.push_back({(uint64_t)lo | ((uint64_t)hi << 32), a_ == lo ? 1u : 2u});
    }
    std::sort(keyed.begin(), keyed.end());
    std::vector<std::pair<uint32_t, uint32_t>> made;
    for (size_t q = 0; q < keyed.size();) {
        uint32_t who = 0;
        size_t r = q;
        while (r < keyed.size() && keyed[r].first == keyed[q].first) who |= keyed[r++].second;
        const uint32_t lo = (uint32_t)keyed[q].first, hi = (uint32_t)(keyed[q].first >> 32);
        made.push_back((who & 1u) ? std::make_pair(lo, hi) : std::make_pair(hi, lo));
        q = r;
    }
    std::sort(made.begin(), made.end());
    *n_connected = (int64_t)made.size();
    if (pairs)
        for (size_t q = 0; q < made.size() && (int64_t)q < cap; ++q) {
            pairs[2 * q] = made[q].first;
            pairs[2 * q + 1] = made[q].second;
        }
    if (made.empty()) return GSIM_OK;
    // (3) gs.outbound on the owned ends, then the connections
    std::vector<uint64_t> pv(made.size());
    std::vector<uint32_t> flat(2 * made.size());
    for (size_t q = 0; q < made.size(); ++q) {
        pv[q] = (uint64_t)made[q].first | ((uint64_t)made[q].second << 32);
        flat[2 * q] = made[q].first;
        flat[2 * q + 1] = made[q].second;
    }
    for (size_t l = 0; l < L; ++l) {
        gsim_handle* h = g->hs[l];
        ShardCtx* s = h->sh;
        (void)hipSetDevice(h->device);
        rc = g->take(h, ensure(h, &s->d_pxin, &s->pxin_cap, (int64_t)pv.size()));
        if (rc) return rc;
        if (stream_copy(h, s->d_pxin, pv.data(), sizeof(uint64_t) * pv.size(), hipMemcpyHostToDevice) != hipSuccess)
            return g->fail(GSIM_EDEVICE, "PX connections upload");
        rc = g->take(h, px_mark_outbound(h, s->d_pxin, (int64_t)pv.size()));
        if (rc) return rc;
    }
    return gsim_group_set_connections(g, flat.data(), (int32_t)made.size(), 1, now);
}

// Join / Leave over the shards (gsim_set_subscriptions per shard, every
// rank with the same list): each shard runs the batch in order over its local
// peers — the owned ones' routers (Join's getPeers and GRAFTs, Leave's PRUNEs),
// the ghosts' announcements — so a later pair sees the earlier ones as on one
// engine; GRAFT/PRUNE to other shards' peers sit in the ghosts' inboxes of
// control round 0 and leave with the heartbeat's control exchange.
int gsim_group_set_subscriptions(gsim_group* g, const uint32_t* pairs, int32_t count, int32_t join, uint64_t tick,
                                 int64_t now)
{
    if (!g || count < 0 || (count > 0 && !pairs)) return GSIM_EINVAL;
    // every pair checked on every process before any shard applies the batch: a
    // rank that held no peer of a bad pair would otherwise go on alone
    const int32_t T = g->hs.empty() ? 64 : std::max(1, g->hs[0]->t);
    for (int32_t q = 0; q < count; ++q)
        if ((int64_t)pairs[2 * q] >= g->N || pairs[2 * q + 1] >= (uint32_t)T || pairs[2 * q + 1] >= 64u)
            return g->fail(GSIM_EINVAL, "subscription pair " + std::to_string(q) + " out of range");
    for (size_t l = 0; l < g->hs.size(); ++l) {
        const std::vector<uint32_t>& gid = g->gid[l];
        std::vector<uint32_t> v;
        for (int32_t q = 0; q < count; ++q) {
            auto it = std::lower_bound(gid.begin(), gid.end(), pairs[2 * q]);
            if (it == gid.end() || *it != pairs[2 * q]) continue;          // not a peer of this shard
            v.push_back((uint32_t)(it - gid.begin()));
            v.push_back(pairs[2 * q + 1]);
        }
        (void)hipSetDevice(g->hs[l]->device);
        const int rc = gsim_set_subscriptions(g->hs[l], v.data(), (int32_t)(v.size() / 2), join, tick, now);
        if (rc) return g->take(g->hs[l], rc);
    }
    for (int32_t q = 0; q < count && !g->sub.empty(); ++q) {
        const uint64_t bit = 1ull << pairs[2 * q + 1];
        if (join) g->sub[pairs[2 * q]] |= bit; else g->sub[pairs[2 * q]] &= ~bit;
    }
    g->router_dirty = true;
    return GSIM_OK;
}

// Totals summed over the shards (every process gets the job's totals).
static int group_sum(gsim_group* g, int (*fn)(gsim_handle*, int64_t*), int n, int64_t* out)
{
    std::vector<int64_t> acc((size_t)n, 0), v((size_t)n);
    int first_err = GSIM_OK;
    for (gsim_handle* h : g->hs) {
        const int rc = fn(h, v.data());
        if (rc && !first_err) { first_err = rc; g->err = "shard: " + h->err; }
        for (int i = 0; i < n; ++i) acc[(size_t)i] += v[(size_t)i];
    }
    if (g->hs.size() < (size_t)g->K) {                  // one shard per process: sum over the ranks
        int64_t* d = nullptr;
        if (hipMalloc((void**)&d, sizeof(int64_t) * (n + 1)) != hipSuccess) return g->fail(GSIM_ENOMEM, "totals scratch");
        acc.push_back(first_err ? 1 : 0);
        (void)stream_copy(g->hs[0], d, acc.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice);
        int rc = g->take_tr(g->tr->allreduce({d}, n + 1, DT_U64, OP_SUM));
        if (!rc) rc = g->take_tr(g->tr->sync());
        (void)stream_copy(g->hs[0], acc.data(), d, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost);
        (void)hipFree(d);
        if (rc) return rc;
        if (acc[(size_t)n] && !first_err) { first_err = GSIM_ERANGE; g->err = "another shard reported an error"; }
    }
    for (int i = 0; i < n; ++i) out[i] = acc[(size_t)i];
    return first_err;
}

int gsim_group_msg_stats(gsim_group* g, int64_t* out4)
{
    if (!g || !out4) return GSIM_EINVAL;
    return group_sum(g, gsim_msg_stats, 4, out4);
}

int gsim_group_gossip_stats(gsim_group* g, int64_t* out4)
{
    if (!g || !out4) return GSIM_EINVAL;
    return group_sum(g, gsim_gossip_stats, 4, out4);
}

int gsim_group_census(gsim_group* g, int64_t* out8)
{
    if (!g || !out8) return GSIM_EINVAL;
    return group_sum(g, gsim_census, 8, out8);
}

int gsim_group_synchronize(gsim_group* g)
{
    if (!g) return GSIM_EINVAL;
    return sync_all(g);
}

int gsim_group_profile(gsim_group* g, int32_t enable)
{
    GROUP_EACH(g, gsim_profile(h, enable));
    return GSIM_OK;
}

int gsim_group_profile_read(gsim_group* g, double* ms, int64_t* launches, int32_t n)
{
    if (!g || n < 0) return GSIM_EINVAL;
    std::vector<double> m((size_t)n);
    std::vector<int64_t> c((size_t)n);
    for (int32_t i = 0; i < n; ++i) { ms[i] = 0.0; launches[i] = 0; }
    for (gsim_handle* h : g->hs) {
        const int rc = gsim_profile_read(h, m.data(), c.data(), n);
        if (rc) return g->take(h, rc);
        for (int32_t i = 0; i < n; ++i) { ms[i] += m[(size_t)i]; launches[i] += c[(size_t)i]; }
    }
    return GSIM_OK;
}


// ---- group readback: the whole network's view of this process's shards ----
// (WithPeerScoreInspect over a sharded network, score.go:152-180, 448-500)

// element size of a field (include/gsim.h gsim_field) and where its peer or
// edge axis is: 0 edge-major [..., E], 1 peer-last [..., N], 2 peer-first [N, ...]
static int field_kind(int32_t f, size_t* es)
{
    switch (f) {
    case GSIM_F_TFLAGS: case GSIM_F_ESTATE: case GSIM_F_CTL: *es = 1; return 0;
    case GSIM_F_SEEN: case GSIM_F_LASTPUT: *es = 4; return 1;
    case GSIM_F_LASTPUB: case GSIM_F_FANOUT_TOPICS: *es = 8; return 2;
    default: *es = 8; return 0;
    }
}

int gsim_group_field_bytes(gsim_group* g, int32_t field, size_t* out)
{
    if (!g || !out || g->hs.empty() || g->bounds.empty()) return GSIM_EINVAL;
    gsim_handle* h = g->hs[0];
    size_t lb = 0;
    int rc = gsim_field_bytes(h, field, &lb);
    if (rc) return g->take(h, rc);
    size_t es = 0;
    const int kind = field_kind(field, &es);
    const size_t per = kind == 0 ? (size_t)h->e * es : (size_t)h->n * es;   // one lead row (or one peer's)
    if (!per) return g->fail(GSIM_ESTATE, "no graph loaded");
    *out = kind == 0 ? lb / per * (size_t)g->E * es : lb / per * (size_t)g->N * es;
    return GSIM_OK;
}

int gsim_group_read_field(gsim_group* g, int32_t field, void* dst, size_t bytes)
{
    if (!g || !dst) return GSIM_EINVAL;
    size_t want = 0;
    int rc = gsim_group_field_bytes(g, field, &want);
    if (rc) return rc;
    if (bytes != want) return g->fail(GSIM_EINVAL, "destination is not the whole network's field size");
    size_t es = 0;
    const int kind = field_kind(field, &es);
    uint8_t* out = static_cast<uint8_t*>(dst);
    std::vector<uint8_t> loc;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        gsim_handle* h = g->hs[l];
        const ShardCtx* sc = h->sh;
        const int k = g->ids[l];
        size_t lb = 0;
        if ((rc = gsim_field_bytes(h, field, &lb))) return g->take(h, rc);
        loc.resize(lb);
        if ((rc = gsim_read_field(h, field, loc.data(), lb))) return g->take(h, rc);
        const int64_t g0 = g->bounds[(size_t)k], np = sc->own_hi - sc->own_lo;
        if (kind == 0) {                         // owned rows: one contiguous run of edges
            const size_t rows = lb / ((size_t)h->e * es), ne = (size_t)(sc->own_e_hi - sc->own_e_lo) * es;
            for (size_t q = 0; q < rows; ++q)
                std::memcpy(out + (q * (size_t)g->E + (size_t)sc->geid_base) * es,
                            loc.data() + (q * (size_t)h->e + (size_t)sc->own_e_lo) * es, ne);
        } else if (kind == 1) {
            const size_t rows = lb / ((size_t)h->n * es);
            for (size_t q = 0; q < rows; ++q)
                std::memcpy(out + (q * (size_t)g->N + (size_t)g0) * es,
                            loc.data() + (q * (size_t)h->n + (size_t)sc->own_lo) * es, (size_t)np * es);
        } else {
            const size_t rowb = lb / (size_t)h->n;
            std::memcpy(out + (size_t)g0 * rowb, loc.data() + (size_t)sc->own_lo * rowb, (size_t)np * rowb);
        }
    }
    return GSIM_OK;
}

int gsim_group_read_scores(gsim_group* g, double* out)
{
    if (!g || !out) return GSIM_EINVAL;
    return gsim_group_read_field(g, GSIM_F_SCORE, out, sizeof(double) * (size_t)g->E);
}

int gsim_group_read_snapshot(gsim_group* g, int64_t obs_lo, int64_t obs_hi, gsim_peer_score_snapshot* peers,
                             gsim_topic_score_snapshot* topics)
{
    if (!g || g->row_ptr.empty()) return GSIM_EINVAL;
    if (obs_lo < 0 || obs_hi > g->N || obs_lo > obs_hi || (!peers && obs_hi > obs_lo))
        return g->fail(GSIM_EINVAL, "observer range out of bounds");
    const int64_t e0 = g->row_ptr[(size_t)obs_lo];
    for (size_t l = 0; l < g->hs.size(); ++l) {
        gsim_handle* h = g->hs[l];
        const ShardCtx* sc = h->sh;
        const int k = g->ids[l];
        const int64_t lo = std::max(obs_lo, g->bounds[(size_t)k]), hi = std::min(obs_hi, g->bounds[(size_t)k + 1]);
        if (lo >= hi) continue;
        const int64_t off = (int64_t)g->row_ptr[(size_t)lo] - e0, T = std::max(1, h->t);
        const int64_t llo = sc->own_lo + (lo - g->bounds[(size_t)k]), lhi = llo + (hi - lo);
        const int rc = gsim_read_snapshot(h, llo, lhi, peers + off, topics ? topics + off * T : nullptr);
        if (rc) return g->take(h, rc);
    }
    return GSIM_OK;
}

// ---- group trace (trace.go:70-530 over a sharded network) ----
// Each shard traces the routers of [peer_lo, peer_hi) it owns, plus the
// events only it knows of at the range's ghosts (TraceRef::on_any: the
// RecvRPC of a copy it pushes to another shard, the SendRPC of an IWANT
// answer from a ghost advertiser, the RecvRPC of an IWANT request to one);
// gsim_group_trace_read merges the shards' events in global ids.
int gsim_group_trace_config(gsim_group* g, uint32_t peer_lo, uint32_t peer_hi, int64_t cap)
{
    if (!g || cap < 0 || peer_lo > peer_hi || (int64_t)peer_hi > g->N) return GSIM_EINVAL;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        gsim_handle* h = g->hs[l];
        const ShardCtx* sc = h->sh;
        if (cap > 0 && !sc->push)
            return g->fail(GSIM_ESTATE, "tracing needs the copy push exchange (GSIM_SHARD_PULL is set)");
        // local ids are in global order: a global range is one local range
        const std::vector<uint32_t>& gid = g->gid[l];
        const uint32_t xlo = (uint32_t)(std::lower_bound(gid.begin(), gid.end(), peer_lo) - gid.begin());
        const uint32_t xhi = (uint32_t)(std::lower_bound(gid.begin(), gid.end(), peer_hi) - gid.begin());
        const uint32_t lo = std::max<uint32_t>(xlo, (uint32_t)sc->own_lo);
        const uint32_t hi = std::max(lo, std::min<uint32_t>(xhi, (uint32_t)sc->own_hi));
        const int rc = trace_config_local(h, lo, hi, xlo, xhi, cap);
        if (rc) return g->take(h, rc);
    }
    return GSIM_OK;
}

int gsim_group_trace_read(gsim_group* g, gsim_trace_event* out, int64_t cap, int64_t* n)
{
    if (!g || !n) return GSIM_EINVAL;
    *n = 0;
    std::vector<int64_t> cnt(g->hs.size(), 0);
    int64_t total = 0;
    for (size_t l = 0; l < g->hs.size(); ++l) {            // the counts first: nothing consumed
        const int rc = gsim_trace_read(g->hs[l], nullptr, 0, &cnt[l]);
        if (rc) return g->take(g->hs[l], rc);
        total += cnt[l];
    }
    *n = total;
    if (!out) return GSIM_OK;
    if (total > cap) return g->fail(GSIM_ERANGE, "output buffer too small for the traced events");
    int64_t off = 0;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        int64_t got = 0;
        const int rc = gsim_trace_read(g->hs[l], out + off, cnt[l], &got);
        if (rc) return g->take(g->hs[l], rc);
        const std::vector<uint32_t>& gid = g->gid[l];
        for (int64_t q = off; q < off + got; ++q) {          // local -> global ids
            out[q].peer = gid[out[q].peer];
            out[q].other = gid[out[q].other];
        }
        off += got;
    }
    *n = off;
    std::sort(out, out + off, [](const gsim_trace_event& a, const gsim_trace_event& b) {
        return std::tie(a.timestamp_ns, a.peer, a.type, a.other, a.reason, a.topic, a.msg_id) <
               std::tie(b.timestamp_ns, b.peer, b.type, b.other, b.reason, b.topic, b.msg_id);
    });
    return GSIM_OK;
}

// ---- the peer gater over a sharded network (peer_gater.go) ----
// Every router's gate lives with its row, on the shard that owns it: the
// copies it receives are gated there -- in place for a copy from an owned
// sender, at the receiving shard's bit apply for a pushed one -- with the
// draw keyed on global ids, so the drops are the single engine's.
int gsim_group_set_peer_gater(gsim_group* g, const gsim_peer_gater_params* p, const double* topic_weights)
{
    if (!g || !p) return GSIM_EINVAL;
    for (gsim_handle* h : g->hs) {
        (void)hipSetDevice(h->device);
        const int rc = gsim_set_peer_gater(h, p, topic_weights);
        if (rc) return g->take(h, rc);
    }
    return GSIM_OK;
}

int gsim_group_gater_throttled(gsim_group* g, int64_t* out)
{
    if (!g || !out) return GSIM_EINVAL;
    return group_sum(g, gsim_gater_throttled, 1, out);
}

int gsim_group_gater_read(gsim_group* g, double* validate, double* throttle, int64_t* last, double* counters4,
                          int32_t* connected, int64_t* expire)
{
    if (!g) return GSIM_EINVAL;
    for (size_t l = 0; l < g->hs.size(); ++l) {
        gsim_handle* h = g->hs[l];
        const ShardCtx* sc = h->sh;
        const int k = g->ids[l];
        const size_t n = (size_t)h->n, e = (size_t)h->e;
        std::vector<double> v(n), t(n), c4(4 * e);
        std::vector<int64_t> la(n), ex(e);
        std::vector<int32_t> co(e);
        const int rc = gsim_gater_read(h, v.data(), t.data(), la.data(), c4.data(), co.data(), ex.data());
        if (rc) return g->take(h, rc);
        const size_t g0 = (size_t)g->bounds[(size_t)k], np = (size_t)(sc->own_hi - sc->own_lo);
        const size_t ge = (size_t)sc->geid_base, ne = (size_t)(sc->own_e_hi - sc->own_e_lo), le = (size_t)sc->own_e_lo;
        if (validate) std::memcpy(validate + g0, v.data() + sc->own_lo, np * 8);
        if (throttle) std::memcpy(throttle + g0, t.data() + sc->own_lo, np * 8);
        if (last) std::memcpy(last + g0, la.data() + sc->own_lo, np * 8);
        if (counters4)
            for (size_t q = 0; q < 4; ++q) std::memcpy(counters4 + q * (size_t)g->E + ge, c4.data() + q * e + le, ne * 8);
        if (connected) std::memcpy(connected + ge, co.data() + le, ne * 4);
        if (expire) std::memcpy(expire + ge, ex.data() + le, ne * 8);
    }
    return GSIM_OK;
}

}  // extern "C"
