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
// Bulk-synchronous restatement.  Round g:
//   k_claim    every accepted copy forwarded in round g-1 does an atomicMin
//              of (0x80000000 | receiving edge) into seen[slot][receiver];
//              committed cells hold a round number < 0x80000000 and are left
//              alone, so the lowest receiving edge claims an unseen cell.
//   k_resolve  each copy re-reads its cell: its own claim -> first delivery
//              (markFirst or markInvalid, joins the frontier); anything else
//              -> duplicate (markDuplicate with validated = the first-seen
//              round's time, or now for a same-round claim).  Counter updates
//              are CAS loops of x -> min(x + 1, cap): every copy applies the
//              same function, so the result is independent of their order.
//   control    rounds 0 and 1 of each heartbeat (GRAFT/PRUNE inbox).
//   k_forward  one wave per frontier entry commits seen = g and appends a
//              copy for every mesh connection except the sender and the origin.
// Lists are compacted with wave ballots (one atomicAdd per wave); list
// lengths stay on the device, kernels use fixed grids with grid-stride loops,
// so a round never synchronizes with the host.
#include <algorithm>
#include <vector>

#include "gsim_internal.h"

namespace gsim {

constexpr uint32_t kUnseen = 0xFFFFFFFFu;
constexpr uint32_t kClaim = 0x80000000u;
constexpr int kListGrid = 2048;   // blocks of the grid-stride list kernels

struct Deliver {
    gsim_msg_config cfg{};
    uint32_t *d_mtopic = nullptr, *d_morigin = nullptr;
    uint8_t* d_minv = nullptr;
    uint32_t* d_seen = nullptr;        // [ring][N]
    int32_t* d_lastput = nullptr;      // [T][N]
    uint32_t* d_f[2][3] = {};          // frontier by round parity: peer, slot, from
    uint32_t* d_a[2][3] = {};          // arrivals by round parity: er, slot, receiver
    uint32_t* d_cnt = nullptr;         // [0..1] frontier lengths, [2..3] arrival lengths, [4] overflow
    unsigned long long* d_stats = nullptr;   // [4]
    gsim_msg* d_pub = nullptr;
    int32_t pub_cap = 0;
    int64_t next_round = -1;           // -1: any
};

struct RoundArgs {
    int64_t N, E;
    int32_t T, ring, R;
    int64_t t0, hb, g, now;
    const uint32_t *row_ptr, *col, *rev;
    const uint8_t* estate;
    const double* score;
    const gsim_topic_score_params* tp;
    double gray;
    uint8_t* tflags;
    double *first, *meshd, *invalid;
    const uint32_t *mtopic, *morigin;
    const uint8_t* minv;
    uint32_t* seen;
    int32_t* lastput;
    const uint32_t *a_er, *a_slot, *a_recv;    // arrivals consumed this round
    uint32_t *f_peer, *f_slot, *f_from;        // frontier of this round
    uint32_t *o_er, *o_slot, *o_recv;          // arrivals produced this round
    uint32_t* cnt;
    int64_t max_frontier, max_arrivals;
    unsigned long long* stats;
};

__device__ __forceinline__ int64_t round_time(const RoundArgs& a, int64_t g)
{
    return a.t0 + (g / a.R) * a.hb + (g % a.R + 1) * a.hb / (a.R + 1);
}

// x -> min(x + 1, cap) on an fp64 counter (markFirst / markDuplicate, score.go
// 919-981); cap = +inf gives invalidMessageDeliveries += 1 (score.go:901-914).
__device__ __forceinline__ void inc_capped(double* p, double cap)
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

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ void k_reset_slots(uint32_t* seen, int64_t N, int32_t ring, const gsim_msg* pub, int32_t count)
{
    const int m = blockIdx.y;
    if (m >= count) return;
    uint32_t* row = seen + (int64_t)(pub[m].id % (uint64_t)ring) * N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x)
        row[i] = kUnseen;
}

__global__ void k_publish(RoundArgs a, const gsim_msg* pub, int32_t count)
{
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= count) return;
    const gsim_msg p = pub[m];
    const uint32_t slot = (uint32_t)(p.id % (uint64_t)a.ring);
    uint32_t* mt = const_cast<uint32_t*>(a.mtopic);
    uint32_t* mo = const_cast<uint32_t*>(a.morigin);
    uint8_t* mi = const_cast<uint8_t*>(a.minv);
    mt[slot] = p.topic;
    mo[slot] = p.origin;
    mi[slot] = p.invalid;
    a.seen[(int64_t)slot * a.N + p.origin] = (uint32_t)a.g;
    a.lastput[(int64_t)p.topic * a.N + p.origin] = (int32_t)(a.g / a.R);
    const uint32_t idx = atomicAdd(&a.cnt[a.g & 1], 1u);
    if ((int64_t)idx >= a.max_frontier) { atomicOr(&a.cnt[4], 1u); return; }
    a.f_peer[idx] = p.origin;
    a.f_slot[idx] = slot;
    a.f_from[idx] = p.origin;
}

// Step 1a: claim unseen cells (lowest receiving edge wins).
__global__ void k_claim(RoundArgs a)
{
    const uint32_t n = min(a.cnt[2 + ((a.g + 1) & 1)], (uint32_t)a.max_arrivals);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t er = a.a_er[i];
        if (a.score[er] < a.gray) continue;
        uint32_t* cell = a.seen + (int64_t)a.a_slot[i] * a.N + a.a_recv[i];
        __hip_atomic_fetch_min(cell, kClaim | er, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Exclusive prefix of v over the 256 threads of a block (4 waves); *total gets
// the block sum.  Must be reached by every thread of the block.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_wt, uint32_t* total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) s_wt[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t x = s_wt[w];
        if (w < wid) wbase += x;
        tot += x;
    }
    *total = tot;
    return wbase + incl - v;
}

constexpr int kResolveItems = 4;   // arrivals per thread per block chunk

// Step 1b: classify every accepted copy and apply the score tracer.  First
// deliveries are appended to the frontier with one global atomic per block
// chunk (256 x kResolveItems copies).
__global__ __launch_bounds__(256) void k_resolve(RoundArgs a)
{
    __shared__ uint32_t s_wt[4];
    __shared__ uint32_t s_base;
    const uint32_t n = min(a.cnt[2 + ((a.g + 1) & 1)], (uint32_t)a.max_arrivals);
    const int lane = threadIdx.x & 63;
    ctp_t tp = const_tp(a.tp);
    const int32_t tick = (int32_t)(a.g / a.R);
    unsigned long long s_acc = 0, s_first = 0, s_gray = 0;
    constexpr uint32_t chunk = 256 * kResolveItems;
    for (uint32_t c0 = blockIdx.x * chunk; c0 < n; c0 += gridDim.x * chunk) {
        uint32_t fr[kResolveItems], fs[kResolveItems], ff[kResolveItems];
        uint32_t fmask = 0;
#pragma unroll
        for (int r = 0; r < kResolveItems; ++r) {
            fr[r] = fs[r] = ff[r] = 0;
            const uint32_t i = c0 + (uint32_t)r * 256 + threadIdx.x;
            if (i >= n) continue;
            const uint32_t er = a.a_er[i];
            const uint32_t slot = a.a_slot[i];
            const uint32_t recv = a.a_recv[i];
            if (a.score[er] < a.gray) {
                s_gray++;
                continue;
            }
            s_acc++;
            const uint32_t c = a.seen[(int64_t)slot * a.N + recv];
            const int32_t t = (int32_t)a.mtopic[slot];
            const bool inv = a.minv[slot] != 0;
            const bool first = c == (kClaim | er);
            const bool scored = (a.estate[er] & GSIM_ES_TRACKED) && tp[t].scored;
            const int64_t te = (int64_t)t * a.E + er;
            if (first) {
                s_first++;
                fmask |= 1u << r;
                fr[r] = recv;
                fs[r] = slot;
                ff[r] = a.col[er];
                if (scored) {
                    if (inv) {
                        inc_capped(&a.invalid[te], __builtin_inf());
                    } else {
                        inc_capped(&a.first[te], tp[t].first_message_deliveries_cap);
                        if (a.tflags[te] & GSIM_TF_IN_MESH)
                            inc_capped(&a.meshd[te], tp[t].mesh_message_deliveries_cap);
                    }
                }
                if (!inv) a.lastput[(int64_t)t * a.N + recv] = tick;
            } else if (scored) {
                if (inv) {
                    inc_capped(&a.invalid[te], __builtin_inf());
                } else if (a.tflags[te] & GSIM_TF_IN_MESH) {
                    const int64_t validated = (c & kClaim) ? a.now : round_time(a, (int64_t)c);
                    if (a.now - validated <= tp[t].mesh_message_deliveries_window_ns)
                        inc_capped(&a.meshd[te], tp[t].mesh_message_deliveries_cap);
                }
            }
        }
        uint32_t total;
        const uint32_t excl = block_excl_scan((uint32_t)__popc(fmask), s_wt, &total);
        if (threadIdx.x == 0) s_base = total ? atomicAdd(&a.cnt[a.g & 1], total) : 0u;
        __syncthreads();
        uint32_t pos = s_base + excl;
#pragma unroll
        for (int r = 0; r < kResolveItems; ++r) {
            if (!((fmask >> r) & 1u)) continue;
            if ((int64_t)pos < a.max_frontier) {
                a.f_peer[pos] = fr[r];
                a.f_slot[pos] = fs[r];
                a.f_from[pos] = ff[r];
            } else {
                atomicOr(&a.cnt[4], 1u);
            }
            ++pos;
        }
        __syncthreads();   // s_wt / s_base reuse
    }
    s_acc = wave_sum_u64(s_acc);
    s_first = wave_sum_u64(s_first);
    s_gray = wave_sum_u64(s_gray);
    if (lane == 0 && (s_acc | s_gray)) {
        atomicAdd(&a.stats[0], s_acc);
        atomicAdd(&a.stats[1], s_first);
        atomicAdd(&a.stats[2], s_acc - s_first);
        atomicAdd(&a.stats[3], s_gray);
    }
}

// Mesh targets of frontier entry q as a lane mask over the sender's row
// (rows of at most 64 connections); lane 0 commits the first-seen round.
// Must be called by a whole wave.
__device__ __forceinline__ uint64_t forward_mask(const RoundArgs& a, uint32_t q, bool commit)
{
    const int lane = threadIdx.x & 63;
    const uint32_t j = a.f_peer[q], slot = a.f_slot[q], from = a.f_from[q];
    if (commit && lane == 0) a.seen[(int64_t)slot * a.N + j] = (uint32_t)a.g;
    const uint32_t t = a.mtopic[slot], origin = a.morigin[slot];
    // receivers reject an invalid message and do not forward it; its
    // origin publishes it regardless
    if (a.minv[slot] && j != origin) return 0;
    const uint32_t b = a.row_ptr[j], deg = a.row_ptr[j + 1] - b;
    const uint32_t e = b + (uint32_t)lane;
    bool ok = false;
    if ((uint32_t)lane < deg) {
        const uint32_t i = a.col[e];
        ok = (a.tflags[(int64_t)t * a.E + e] & GSIM_TF_MESH) && (a.estate[e] & GSIM_ES_CONNECTED) && i != from &&
             i != origin;
    }
    return __ballot(ok);
}

// Step 3: commit first-seen rounds and forward to the mesh.  A block takes 256
// frontier entries (64 per wave): pass 1 builds each entry's target mask,
// one global atomic reserves the block's output range, pass 2 writes it.
__global__ __launch_bounds__(256) void k_forward(RoundArgs a)
{
    __shared__ uint32_t s_wt[4];
    __shared__ uint32_t s_base;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // the lists of round g+1's parity were consumed by round g-1 / g
        a.cnt[(a.g + 1) & 1] = 0;
        a.cnt[2 + ((a.g + 1) & 1)] = 0;
    }
    const uint32_t n = min(a.cnt[a.g & 1], (uint32_t)a.max_frontier);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t c0 = blockIdx.x * 256; c0 < n; c0 += gridDim.x * 256) {
        const uint32_t w0 = c0 + (uint32_t)wid * 64;
        uint64_t my_mask = 0;
        for (int q = 0; q < 64; ++q) {
            if (w0 + q >= n) break;
            const uint64_t m = forward_mask(a, w0 + q, true);
            if (lane == q) my_mask = m;
        }
        uint32_t total;
        const uint32_t excl = block_excl_scan((uint32_t)__popcll(my_mask), s_wt, &total);
        if (threadIdx.x == 0) s_base = total ? atomicAdd(&a.cnt[2 + (a.g & 1)], total) : 0u;
        __syncthreads();
        const uint32_t base = s_base;
        for (int q = 0; q < 64; ++q) {
            const uint32_t idx = w0 + q;
            if (idx >= n) break;
            const uint64_t m = __shfl(my_mask, q, 64);
            if (!m) continue;
            const uint32_t off = base + __shfl(excl, q, 64);
            if ((m >> lane) & 1ull) {
                const uint32_t j = a.f_peer[idx];
                const uint32_t e = a.row_ptr[j] + (uint32_t)lane;
                const uint32_t pos = off + (uint32_t)__popcll(m & ((1ull << lane) - 1));
                if ((int64_t)pos < a.max_arrivals) {
                    a.o_er[pos] = a.rev[e];
                    a.o_slot[pos] = a.f_slot[idx];
                    a.o_recv[pos] = a.col[e];
                } else {
                    atomicOr(&a.cnt[4], 1u);
                }
            }
        }
        __syncthreads();   // s_wt / s_base reuse
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
    f(d->d_mtopic); f(d->d_morigin); f(d->d_minv); f(d->d_seen); f(d->d_lastput);
    for (int p = 0; p < 2; ++p)
        for (int k = 0; k < 3; ++k) { f(d->d_f[p][k]); f(d->d_a[p][k]); }
    f(d->d_cnt); f(d->d_stats); f(d->d_pub);
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
    if (f == GSIM_F_SEEN) { *r = {d->d_seen, (size_t)d->cfg.ring * (size_t)h->n * 4}; return true; }
    if (f == GSIM_F_LASTPUT) { *r = {d->d_lastput, (size_t)std::max(1, h->t) * (size_t)h->n * 4}; return true; }
    return false;
}

static RoundArgs make_round_args(gsim_handle* h, int64_t g)
{
    Deliver* d = h->dl;
    RoundArgs a{};
    a.N = h->n; a.E = h->e; a.T = h->t; a.ring = d->cfg.ring; a.R = d->cfg.rounds;
    a.t0 = d->cfg.t0_ns; a.hb = d->cfg.heartbeat_ns; a.g = g;
    a.now = a.t0 + (g / a.R) * a.hb + (g % a.R + 1) * a.hb / (a.R + 1);
    a.row_ptr = h->d_row_ptr; a.col = h->d_col; a.rev = h->d_rev;
    a.estate = h->d_estate; a.score = h->d_score; a.tp = h->d_tp; a.gray = h->th.graylist_threshold;
    a.tflags = h->d_tflags; a.first = h->d_first; a.meshd = h->d_meshd; a.invalid = h->d_invalid;
    a.mtopic = d->d_mtopic; a.morigin = d->d_morigin; a.minv = d->d_minv;
    a.seen = d->d_seen; a.lastput = d->d_lastput;
    const int pin = (int)((g + 1) & 1), pout = (int)(g & 1);
    a.a_er = d->d_a[pin][0]; a.a_slot = d->d_a[pin][1]; a.a_recv = d->d_a[pin][2];
    a.o_er = d->d_a[pout][0]; a.o_slot = d->d_a[pout][1]; a.o_recv = d->d_a[pout][2];
    a.f_peer = d->d_f[pout][0]; a.f_slot = d->d_f[pout][1]; a.f_from = d->d_f[pout][2];
    a.cnt = d->d_cnt;
    a.max_frontier = d->cfg.max_frontier; a.max_arrivals = d->cfg.max_arrivals;
    a.stats = d->d_stats;
    return a;
}

extern "C" {

int gsim_msgs_init(gsim_handle* h, const gsim_msg_config* cfg)
{
    if (!h || !cfg) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (h->e == 0) { h->err = "no graph loaded"; return GSIM_ESTATE; }
    if (cfg->ring <= 0 || cfg->rounds < 2 || cfg->heartbeat_ns <= 0 || cfg->max_frontier <= 0 ||
        cfg->max_arrivals <= 0 || cfg->max_frontier > 0x7FFFFFFF || cfg->max_arrivals > 0x7FFFFFFF) {
        h->err = "invalid message configuration";
        return GSIM_EINVAL;
    }
    (void)hipStreamSynchronize(h->stream);
    free_deliver(h);
    Deliver* d = new Deliver();
    d->cfg = *cfg;
    const size_t ring = (size_t)cfg->ring, N = (size_t)h->n, T = (size_t)std::max(1, h->t);
    hipError_t e = hipSuccess;
    auto A = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, std::max<size_t>(bytes, 4));
        if (e == hipSuccess) h->bytes_allocated += bytes;
    };
    A((void**)&d->d_mtopic, ring * 4);
    A((void**)&d->d_morigin, ring * 4);
    A((void**)&d->d_minv, ring);
    A((void**)&d->d_seen, ring * N * 4);
    A((void**)&d->d_lastput, T * N * 4);
    for (int p = 0; p < 2; ++p)
        for (int k = 0; k < 3; ++k) {
            A((void**)&d->d_f[p][k], (size_t)cfg->max_frontier * 4);
            A((void**)&d->d_a[p][k], (size_t)cfg->max_arrivals * 4);
        }
    A((void**)&d->d_cnt, 8 * 4);
    A((void**)&d->d_stats, 4 * 8);
    if (e != hipSuccess) {
        dl_free(d);
        h->err = std::string("message ring allocation: ") + hipGetErrorString(e);
        return e == hipErrorOutOfMemory ? GSIM_ENOMEM : GSIM_EDEVICE;
    }
    h->dl = d;
    e = hipMemsetAsync(d->d_seen, 0xFF, ring * N * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_lastput, 0xFF, T * N * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_mtopic, 0, ring * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_morigin, 0, ring * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_minv, 0, ring, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_cnt, 0, 8 * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_stats, 0, 4 * 8, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return hip_check(h, e, "gsim_msgs_init");
}

int gsim_publish(gsim_handle* h, const gsim_msg* msgs, int32_t count, int64_t round)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    if (count < 0 || (count > 0 && !msgs) || round < 0) return GSIM_EINVAL;
    if (count == 0) return GSIM_OK;
    if (d->next_round >= 0 && round != d->next_round) {
        h->err = "messages must be published for the next round";
        return GSIM_ESTATE;
    }
    std::vector<uint32_t> slots((size_t)count);
    for (int32_t m = 0; m < count; ++m) {
        if (msgs[m].topic >= (uint32_t)std::max(1, h->t) || (int64_t)msgs[m].origin >= h->n) {
            h->err = "message topic or origin out of range";
            return GSIM_EINVAL;
        }
        slots[(size_t)m] = (uint32_t)(msgs[m].id % (uint64_t)d->cfg.ring);
    }
    std::sort(slots.begin(), slots.end());
    if (std::adjacent_find(slots.begin(), slots.end()) != slots.end()) {
        h->err = "two messages of one publish batch share a ring slot";
        return GSIM_EINVAL;
    }
    hipError_t e = hipSuccess;
    if (count > d->pub_cap) {
        if (d->d_pub) { (void)hipStreamSynchronize(h->stream); (void)hipFree(d->d_pub); d->d_pub = nullptr; }
        const int32_t cap = std::max(count, 256);
        e = hipMalloc((void**)&d->d_pub, sizeof(gsim_msg) * (size_t)cap);
        if (e != hipSuccess) { d->pub_cap = 0; return hip_check(h, e, "hipMalloc publish"); }
        d->pub_cap = cap;
    }
    e = hipMemcpyAsync(d->d_pub, msgs, sizeof(gsim_msg) * (size_t)count, hipMemcpyHostToDevice, h->stream);
    if (e != hipSuccess) return hip_check(h, e, "publish upload");
    ProfScope ps(h, GSIM_K_PUBLISH);
    const int64_t per_block = 256 * 16;
    const int gx = (int)std::min<int64_t>((h->n + per_block - 1) / per_block, 1024);
    hipLaunchKernelGGL(k_reset_slots, dim3(std::max(gx, 1), count), dim3(256), 0, h->stream, d->d_seen, h->n,
                       d->cfg.ring, (const gsim_msg*)d->d_pub, count);
    RoundArgs a = make_round_args(h, round);
    hipLaunchKernelGGL(k_publish, dim3((count + 255) / 256), dim3(256), 0, h->stream, a,
                       (const gsim_msg*)d->d_pub, count);
    d->next_round = round;
    return hip_check(h, hipGetLastError(), "k_publish");
}

int gsim_round(gsim_handle* h, int64_t round)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    if (round < 0 || round >= 0x7FFFFFFF) return GSIM_ERANGE;
    if (d->next_round >= 0 && round != d->next_round) {
        h->err = "rounds must be consecutive";
        return GSIM_ESTATE;
    }
    if (h->max_degree > 64) {
        h->err = "propagation kernels support rows of at most 64 connections in this build";
        return GSIM_ERANGE;
    }
    RoundArgs a = make_round_args(h, round);
    {
        ProfScope ps(h, GSIM_K_CLAIM);
        hipLaunchKernelGGL(k_claim, dim3(kListGrid), dim3(256), 0, h->stream, a);
    }
    {
        ProfScope ps(h, GSIM_K_RESOLVE);
        hipLaunchKernelGGL(k_resolve, dim3(kListGrid), dim3(256), 0, h->stream, a);
    }
    int rc = hip_check(h, hipGetLastError(), "k_claim/k_resolve");
    if (rc) return rc;
    const int32_t r = (int32_t)(round % d->cfg.rounds);
    if (r < 2) {
        // rounds >= 2 of a heartbeat have an empty control inbox: handling
        // PRUNE replies (round 1) emits nothing
        rc = gsim_handle_control(h, r, a.now);
        if (rc) return rc;
    }
    {
        ProfScope ps(h, GSIM_K_FORWARD);
        hipLaunchKernelGGL(k_forward, dim3(kListGrid), dim3(256), 0, h->stream, a);
    }
    d->next_round = round + 1;
    return hip_check(h, hipGetLastError(), "k_forward");
}

int gsim_msg_stats(gsim_handle* h, int64_t* out4)
{
    if (!h || !out4) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    unsigned long long s[4];
    uint32_t ovf = 0;
    hipError_t e = hipMemcpyAsync(s, d->d_stats, sizeof(s), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&ovf, d->d_cnt + 4, 4, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_msg_stats");
    for (int k = 0; k < 4; ++k) out4[k] = (int64_t)s[k];
    if (ovf) {
        h->err = "a round overflowed max_frontier or max_arrivals";
        return GSIM_ERANGE;
    }
    return GSIM_OK;
}

}  // extern "C"
