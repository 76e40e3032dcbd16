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
// message state: seen[slot][peer] = first-seen round, so the forwarding
// frontier of round g-1 is {j : seen[m][j] == g-1} and no per-copy list is
// ever materialized.  Round g:
//   k_send    one wave per 64 consecutive senders, for every slot active in
//             round g-1 (a coalesced load of seen[m][j0..j0+63] per slot):
//             each frontier sender walks its row with a lane group, and for
//             every mesh target evaluates AcceptFrom, loads the receiver's
//             seen cell and applies the score tracer to the RECEIVER's record
//             of the sender, which in record order sits at the
//             sender's own edge index: the counter traffic is coalesced along
//             the sender's row.  A copy to a cell already committed is a
//             duplicate (validated = its first-seen round); a copy to an
//             uncommitted cell claims it with an atomicMin of
//             (0x80000000 | edge): the lowest edge, i.e. the lowest sender,
//             wins.  Every same-round copy, first or duplicate, has
//             validated = now and therefore the same counter update; only
//             firstMessageDeliveries needs the winner.
//   k_commit  one wave per 64 consecutive receivers, for the same slots: a
//             claimed cell commits seen = g and from = the winner, and the
//             winner's record gets markFirstMessageDelivery's P2 credit.
//   control   rounds 0 and 1 of each heartbeat (GRAFT/PRUNE inbox).
// Counter updates are plain read-modify-writes: in k_send a record (receiver
// i, sender j) is only touched by the lanes that walk j's row, always the
// same lanes of the same wave; in k_commit only by receiver i's lane.
#include <algorithm>
#include <vector>

#include "gsim_internal.h"

namespace gsim {

constexpr uint32_t kUnseen = 0xFFFFFFFFu;
constexpr uint32_t kClaim = 0x80000000u;
constexpr int kMaxRing = 8192;     // active-slot list lives in LDS (u16)

struct Deliver {
    gsim_msg_config cfg{};
    uint32_t *d_mtopic = nullptr, *d_morigin = nullptr;
    uint8_t* d_minv = nullptr;
    uint32_t* d_seen = nullptr;        // [ring][N] first-seen round
    uint32_t* d_from = nullptr;        // [ring][N] sender of the first copy
    int32_t* d_lastput = nullptr;      // [T][N]
    uint32_t* d_nfirst = nullptr;      // [2][ring] first receptions per slot, by round parity
    unsigned long long* d_stats = nullptr;   // [4]
    gsim_msg* d_pub = nullptr;
    int32_t pub_cap = 0;
    int64_t next_round = -1;           // -1: any
};

struct RoundArgs {
    int64_t N, E;
    int32_t T, ring, R;
    int64_t t0, hb, g, now;
    const uint32_t *row_ptr, *col, *owner;
    const uint8_t* rstate;     // router connected bit, edge order
    const uint8_t* mflags;     // router mesh bits, edge order
    const uint8_t* acc;        // AcceptFrom verdicts, record order
    const uint8_t* estate;     // record order
    const uint8_t* tflags;     // score bits, record order
    const gsim_topic_score_params* tp;
    double *first, *meshd, *invalid;
    uint32_t *mtopic, *morigin;
    uint8_t* minv;
    uint32_t *seen, *from;
    int32_t* lastput;
    const uint32_t* nfirst_prev;   // slots with a frontier in round g-1
    uint32_t* nfirst_cur;          // first receptions of round g
    unsigned long long* stats;
};

__device__ __forceinline__ int64_t round_time(const RoundArgs& a, int64_t g)
{
    return a.t0 + (g / a.R) * a.hb + (g % a.R + 1) * a.hb / (a.R + 1);
}

// x -> min(x + 1, cap) (markFirst / markDuplicate, score.go:919-981)
__device__ __forceinline__ void inc_capped(double* p, double cap)
{
    double x = *p + 1.0;
    if (x > cap) x = cap;
    *p = x;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Ordered list of the slots that had first receptions (or a publication) in
// round g-1, built by wave 0 into LDS; every thread of the block must call it.
__device__ __forceinline__ int active_slots(const RoundArgs& a, uint16_t* s_act, int* s_n)
{
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        int n = 0;
        for (int m0 = 0; m0 < a.ring; m0 += 64) {
            const int m = m0 + lane;
            const bool act = m < a.ring && a.nfirst_prev[m] != 0;
            const uint64_t b = __ballot(act);
            if (act) s_act[n + __popcll(b & ((1ull << lane) - 1))] = (uint16_t)m;
            n += __popcll(b);
        }
        if (lane == 0) *s_n = n;
    }
    __syncthreads();
    return *s_n;
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
    a.mtopic[slot] = p.topic;
    a.morigin[slot] = p.origin;
    a.minv[slot] = p.invalid;
    a.seen[(int64_t)slot * a.N + p.origin] = (uint32_t)a.g;
    a.from[(int64_t)slot * a.N + p.origin] = p.origin;
    a.lastput[(int64_t)p.topic * a.N + p.origin] = (int32_t)(a.g / a.R);
    a.nfirst_cur[slot] = 1;   // the origin forwards in round g+1
}

// Round g, step 1: every frontier sender of round g-1 forwards to its mesh.
// W = lanes per row (power of two >= the longest row); group q of a wave
// always walks the senders j0 + q*W .. j0 + q*W + W-1.
template <int W>
__global__ __launch_bounds__(256) void k_send(RoundArgs a)
{
    __shared__ uint16_t s_act[kMaxRing];
    __shared__ int s_n;
    const int nact = a.g > 0 ? active_slots(a, s_act, &s_n) : 0;   // round 0 has no predecessor
    const int lane = threadIdx.x & 63;
    const int64_t j0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
    if (j0 >= a.N) return;
    const int64_t jl = j0 + lane;
    const bool vj = jl < a.N;
    const int grp = lane / W, gl = lane % W;
    const uint64_t gmask = (W == 64) ? ~0ull : (((1ull << W) - 1) << (grp * W));
    const ctp_t tpa = const_tp(a.tp);
    const uint32_t gprev = (uint32_t)(a.g - 1);
    unsigned long long n_acc = 0, n_gray = 0;
    for (int k = 0; k < nact; ++k) {
        const uint32_t m = s_act[k];
        const int64_t row_m = (int64_t)m * a.N;
        const uint32_t origin = a.morigin[m];
        const bool inv = a.minv[m] != 0;
        const uint32_t sv = vj ? a.seen[row_m + jl] : kUnseen;
        // receivers reject an invalid message and do not forward it; its
        // origin publishes it regardless
        const bool fr = sv == gprev && (!inv || (uint32_t)jl == origin);
        const uint64_t mask = __ballot(fr);
        if (!mask) continue;
        const uint32_t from_l = fr ? a.from[row_m + jl] : 0u;
        const int32_t t = (int32_t)a.mtopic[m];
        const ctp_t tp = tpa + t;
        const bool scored_t = tp->scored != 0;
        const int64_t window = tp->mesh_message_deliveries_window_ns;
        const double mcap = tp->mesh_message_deliveries_cap;
        const int64_t plane = (int64_t)t * a.E;
        uint64_t gm = mask & gmask;
        while (__ballot(gm != 0)) {
            int b = -1;
            if (gm) { b = __ffsll((long long)gm) - 1; gm &= gm - 1; }
            const uint32_t fromj = __shfl(from_l, b < 0 ? lane : b, 64);
            if (b < 0) continue;
            const uint32_t j = (uint32_t)(j0 + b);
            const uint32_t beg = a.row_ptr[j];
            const uint32_t deg = a.row_ptr[j + 1] - beg;
            if ((uint32_t)gl >= deg) continue;
            const uint32_t e = beg + (uint32_t)gl;
            const uint32_t i = a.col[e];
            if (!(a.mflags[plane + e] & GSIM_TF_MESH) || !(a.rstate[e] & GSIM_ES_CONNECTED) || i == fromj ||
                i == origin)
                continue;
            if (!a.acc[e]) { n_gray++; continue; }     // AcceptFrom: graylisted sender
            n_acc++;
            uint32_t* cell = a.seen + row_m + i;
            const uint32_t c = *cell;
            const bool old = c < kClaim;                 // committed in an earlier round
            if (!old) __hip_atomic_fetch_min(cell, kClaim | e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!scored_t || !(a.estate[e] & GSIM_ES_TRACKED)) continue;
            const int64_t ir = plane + e;
            if (inv) {                                   // markInvalidMessageDelivery
                a.invalid[ir] = a.invalid[ir] + 1.0;
                continue;
            }
            if (!(a.tflags[ir] & GSIM_TF_IN_MESH)) continue;
            // markDuplicateMessageDelivery's window test; a same-round copy
            // (first or duplicate) has validated = now
            const bool in_window = old ? (a.now - round_time(a, (int64_t)c) <= window) : (window >= 0);
            if (in_window) inc_capped(&a.meshd[ir], mcap);
        }
    }
    n_acc = wave_sum_u64(n_acc);
    n_gray = wave_sum_u64(n_gray);
    if (lane == 0 && (n_acc | n_gray)) {
        atomicAdd(&a.stats[0], n_acc);
        atomicAdd(&a.stats[2], n_acc);          // k_commit moves the firsts out
        atomicAdd(&a.stats[3], n_gray);
    }
}

// Round g, step 2: commit every claimed cell (markSeen) and credit the
// winner's first delivery (markFirstMessageDelivery, score.go:919-946).
__global__ __launch_bounds__(256) void k_commit(RoundArgs a)
{
    __shared__ uint16_t s_act[kMaxRing];
    __shared__ int s_n;
    const int nact = a.g > 0 ? active_slots(a, s_act, &s_n) : 0;
    const int lane = threadIdx.x & 63;
    const int64_t i0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
    if (i0 >= a.N) return;
    const int64_t i = i0 + lane;
    const bool vi = i < a.N;
    const ctp_t tpa = const_tp(a.tp);
    const int32_t tick = (int32_t)(a.g / a.R);
    unsigned long long n_first = 0;
    for (int k = 0; k < nact; ++k) {
        const uint32_t m = s_act[k];
        const int64_t cell = (int64_t)m * a.N + i;
        const uint32_t c = vi ? a.seen[cell] : kUnseen;
        const bool claimed = c != kUnseen && (c & kClaim);
        const uint64_t cm = __ballot(claimed);
        if (!cm) continue;
        if (lane == 0) atomicAdd(&a.nfirst_cur[m], (uint32_t)__popcll(cm));
        if (!claimed) continue;
        n_first++;
        const uint32_t ew = c & ~kClaim;           // winning edge = the receiver's record of the sender
        const int32_t t = (int32_t)a.mtopic[m];
        const bool inv = a.minv[m] != 0;
        a.seen[cell] = (uint32_t)a.g;
        a.from[cell] = a.owner[ew];
        if (inv) continue;                          // RejectMessage: counted by k_send
        a.lastput[(int64_t)t * a.N + i] = tick;     // mcache.Put
        const ctp_t tp = tpa + t;
        if (!tp->scored || !(a.estate[ew] & GSIM_ES_TRACKED)) continue;
        const int64_t ir = (int64_t)t * a.E + ew;
        inc_capped(&a.first[ir], tp->first_message_deliveries_cap);
        // with a negative window k_send credits no same-round copy; the first
        // delivery is credited regardless of the window
        if (tp->mesh_message_deliveries_window_ns < 0 && (a.tflags[ir] & GSIM_TF_IN_MESH))
            inc_capped(&a.meshd[ir], tp->mesh_message_deliveries_cap);
    }
    n_first = wave_sum_u64(n_first);
    if (lane == 0 && n_first) {
        atomicAdd(&a.stats[1], n_first);
        atomicAdd(&a.stats[2], 0ull - n_first);   // duplicates = accepted - first
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
    f(d->d_mtopic); f(d->d_morigin); f(d->d_minv); f(d->d_seen); f(d->d_from); f(d->d_lastput);
    f(d->d_nfirst); f(d->d_stats); f(d->d_pub);
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
    a.row_ptr = h->d_row_ptr; a.col = h->d_col; a.owner = h->d_owner;
    a.rstate = h->d_rstate; a.mflags = h->d_mflags; a.acc = h->d_acc;
    a.estate = h->d_estate; a.tflags = h->d_tflags; a.tp = h->d_tp;
    a.first = h->d_first; a.meshd = h->d_meshd; a.invalid = h->d_invalid;
    a.mtopic = d->d_mtopic; a.morigin = d->d_morigin; a.minv = d->d_minv;
    a.seen = d->d_seen; a.from = d->d_from; a.lastput = d->d_lastput;
    const size_t ring = (size_t)d->cfg.ring;
    a.nfirst_prev = d->d_nfirst + (size_t)((g + 1) & 1) * ring;
    a.nfirst_cur = d->d_nfirst + (size_t)(g & 1) * ring;
    a.stats = d->d_stats;
    return a;
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
    if (h->e >= (int64_t)kClaim) { h->err = "too many edges for the seen-set claim encoding"; return GSIM_ERANGE; }
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
    A((void**)&d->d_from, ring * N * 4);
    A((void**)&d->d_lastput, T * N * 4);
    A((void**)&d->d_nfirst, 2 * ring * 4);
    A((void**)&d->d_stats, 4 * 8);
    if (e != hipSuccess) {
        dl_free(d);
        h->err = std::string("message ring allocation: ") + hipGetErrorString(e);
        return e == hipErrorOutOfMemory ? GSIM_ENOMEM : GSIM_EDEVICE;
    }
    h->dl = d;
    e = hipMemsetAsync(d->d_seen, 0xFF, ring * N * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_from, 0, ring * N * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_lastput, 0xFF, T * N * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_mtopic, 0, ring * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_morigin, 0, ring * 4, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_minv, 0, ring, h->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d->d_nfirst, 0, 2 * ring * 4, h->stream);
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
    if (round < 0 || round >= 0x7FFFFFFF) { h->err = "round out of range [0, 2^31-1)"; return GSIM_ERANGE; }
    if (d->next_round >= 0 && round != d->next_round) {
        h->err = "rounds must be consecutive";
        return GSIM_ESTATE;
    }
    if (h->max_degree > 64) {
        h->err = "propagation kernels support rows of at most 64 connections in this build";
        return GSIM_ERANGE;
    }
    int rc = 0;
    {
        ProfScope ps(h, GSIM_K_ACCEPT);
        rc = refresh_accept(h);
        if (rc) return rc;
    }
    RoundArgs a = make_round_args(h, round);
    const int64_t waves = (h->n + 63) / 64;
    const int grid = (int)std::max<int64_t>((waves + 3) / 4, 1);
    {
        ProfScope ps(h, GSIM_K_SEND);
        if (h->max_degree <= 16)
            hipLaunchKernelGGL(k_send<16>, dim3(grid), dim3(256), 0, h->stream, a);
        else if (h->max_degree <= 32)
            hipLaunchKernelGGL(k_send<32>, dim3(grid), dim3(256), 0, h->stream, a);
        else
            hipLaunchKernelGGL(k_send<64>, dim3(grid), dim3(256), 0, h->stream, a);
    }
    {
        ProfScope ps(h, GSIM_K_COMMIT);
        hipLaunchKernelGGL(k_commit, dim3(grid), dim3(256), 0, h->stream, a);
        // the counters of round g+1 were last read as "previous" by round g
        hipError_t e = hipMemsetAsync(d->d_nfirst + (size_t)((round + 1) & 1) * (size_t)d->cfg.ring, 0,
                                      (size_t)d->cfg.ring * 4, h->stream);
        if (e != hipSuccess) return hip_check(h, e, "nfirst reset");
    }
    rc = hip_check(h, hipGetLastError(), "k_send/k_commit");
    if (rc) return rc;
    const int32_t r = (int32_t)(round % d->cfg.rounds);
    if (r < 2) {
        // rounds >= 2 of a heartbeat have an empty control inbox: handling
        // PRUNE replies (round 1) emits nothing
        rc = gsim_handle_control(h, r, a.now);
        if (rc) return rc;
    }
    d->next_round = round + 1;
    return GSIM_OK;
}

int gsim_msg_stats(gsim_handle* h, int64_t* out4)
{
    if (!h || !out4) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    Deliver* d = h->dl;
    if (!d) { h->err = "gsim_msgs_init not called"; return GSIM_ESTATE; }
    unsigned long long s[4];
    hipError_t e = hipMemcpyAsync(s, d->d_stats, sizeof(s), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_msg_stats");
    for (int k = 0; k < 4; ++k) out4[k] = (int64_t)s[k];
    return GSIM_OK;
}

}  // extern "C"
