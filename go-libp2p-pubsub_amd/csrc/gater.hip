// gater.hip — the peer gater of every router (peer_gater.go; SURVEY.md §8(f)
// row 3): random-early-drop AcceptFrom over per-IP delivery statistics.
//
// Reference: PeerGaterParams + validate (peer_gater.go:31-111), decayStats
// (207-241), getPeerStats / getIPStats / getPeerIP (243-318), AcceptFrom
// (320-363), the RawTracer hooks (366-443); gossipsub.go:598-609 puts the
// gate behind the graylist.
//
// Layout (all device arrays):
//   per router i        validate, throttle (f64), lastThrottle (i64), and the
//                       round's event counts (u32) and throttle flag
//   per connection e    (edge order, i = the row's owner) rep[e]: the row
//                       position that holds the stats of col[e]'s IP at i —
//                       the lowest position with the same IP key; the IP
//                       group's deliver / duplicate / ignore / reject (f64),
//                       connected (i32), expire (i64) and the round's
//                       event counts live at that position
//   per record r        gq[r] = rep[rev[r]]: the delivery kernels, which
//                       walk records in the sender's row, find the group of
//                       receiver i's stats about the sender in one load
// A round's events are integer counts added atomically by the delivery
// kernels (copies: duplicate / bad signature; the claim winner converts its
// duplicate into its verdict's event at commit) and folded into the f64
// counters after the commit (gater_fold), so the result does not depend on
// the order the copies were handled in; the oracle (oracle/oracle_gater.c)
// folds the same counts at the end of each round.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "gsim_internal.h"

namespace gsim {

struct Gater {
    gsim_peer_gater_params p{};
    uint32_t* rep = nullptr;                  // [E] edge order
    uint32_t* gq = nullptr;                   // [E] record order
    double *del = nullptr, *dup = nullptr, *ign = nullptr, *rej = nullptr;   // [E] at reps
    int32_t* con = nullptr;
    int64_t* exp = nullptr;
    unsigned long long* a_del = nullptr;      // [E] 2^-16 units
    uint32_t *a_dup = nullptr, *a_ign = nullptr, *a_rej = nullptr;
    double *val = nullptr, *thr = nullptr;    // [N]
    int64_t* last = nullptr;
    uint32_t *a_val = nullptr, *a_thr = nullptr;
    uint8_t* a_last = nullptr;
    uint8_t* act = nullptr;                   // [N] the gate may throttle this round
    unsigned long long* tw = nullptr;         // [T] delivery weights, 2^-16 units
    unsigned long long* n_thr = nullptr;      // [1] copies dropped
    int64_t fold_round = -1;                  // events of this round are not folded yet
};

namespace {

constexpr int64_t kNever = INT64_MIN;        // lastThrottle before any throttle (time.Time{})
constexpr uint32_t kNoIp = 0xFFFFFFFFu;      // getPeerIP's "<unknown>"

__device__ __forceinline__ uint32_t ip_key(const uint32_t* ip_ptr, const uint32_t* ip_ids, uint32_t p)
{
    if (!ip_ptr || ip_ptr[p] == ip_ptr[p + 1]) return kNoIp;
    return ip_ids[ip_ptr[p]];
}

// rep[e]: the lowest position of e's row whose peer has col[e]'s IP key; the
// connected count of every group (AddPeer of the connections that exist)
__global__ __launch_bounds__(256) void k_gater_groups(const uint32_t* row_ptr, const uint32_t* col,
                                                      const uint32_t* owner, const uint32_t* ip_ptr,
                                                      const uint32_t* ip_ids, const uint8_t* rstate, int64_t E,
                                                      uint32_t* rep, int32_t* con)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) {
        const uint32_t o = owner[e];
        const uint32_t k = ip_key(ip_ptr, ip_ids, col[e]);
        uint32_t r = (uint32_t)e;
        for (uint32_t f = row_ptr[o]; f < (uint32_t)e; ++f)
            if (ip_key(ip_ptr, ip_ids, col[f]) == k) { r = f; break; }
        rep[e] = r;
        if (rstate[e] & GSIM_ES_CONNECTED) atomicAdd(&con[r], 1);
    }
}

__global__ __launch_bounds__(256) void k_gater_gq(const uint32_t* rep, const uint32_t* rev, int64_t E, uint32_t* gq)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < E; r += stride) gq[r] = rep[rev[r]];
}

// AcceptFrom's preamble (peer_gater.go:327-343) at round time now
__global__ __launch_bounds__(256) void k_gater_active(const double* val, const double* thr, const int64_t* last,
                                                      int64_t N, int64_t now, int64_t quiet, double threshold,
                                                      uint8_t* act)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += stride) {
        bool a = true;
        if (last[i] == kNever || now - last[i] > quiet) a = false;
        else if (thr[i] == 0) a = false;
        else if (val[i] != 0 && thr[i] / val[i] < threshold) a = false;
        act[i] = a ? 1 : 0;
    }
}

// the round's events into the counters
__global__ __launch_bounds__(256) void k_gater_fold(Gater g, int64_t N, int64_t E, int64_t now)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < (N > E ? N : E); x += stride) {
        if (x < N) {
            if (g.a_val[x]) { g.val[x] += (double)g.a_val[x]; g.a_val[x] = 0; }
            if (g.a_thr[x]) { g.thr[x] += (double)g.a_thr[x]; g.a_thr[x] = 0; }
            if (g.a_last[x]) { g.last[x] = now; g.a_last[x] = 0; }
        }
        if (x >= E) continue;
        if (g.a_del[x]) { g.del[x] += (double)g.a_del[x] * (1.0 / 65536.0); g.a_del[x] = 0; }
        if (g.a_dup[x]) { g.dup[x] += (double)g.a_dup[x]; g.a_dup[x] = 0; }
        if (g.a_ign[x]) { g.ign[x] += (double)g.a_ign[x]; g.a_ign[x] = 0; }
        if (g.a_rej[x]) { g.rej[x] += (double)g.a_rej[x]; g.a_rej[x] = 0; }
    }
}

__device__ __forceinline__ double decay1(double x, double d, double dtz)
{
    x *= d;
    return x < dtz ? 0.0 : x;
}

// decayStats (peer_gater.go:207-241)
__global__ __launch_bounds__(256) void k_gater_decay(Gater g, int64_t N, int64_t E, int64_t now)
{
    const double dtz = g.p.decay_to_zero, gd = g.p.global_decay, sd = g.p.source_decay;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < (N > E ? N : E); x += stride) {
        if (x < N) {
            g.val[x] = decay1(g.val[x], gd, dtz);
            g.thr[x] = decay1(g.thr[x], gd, dtz);
        }
        if (x >= E || g.rep[x] != (uint32_t)x) continue;
        if (g.con[x] > 0) {
            g.del[x] = decay1(g.del[x], sd, dtz);
            g.dup[x] = decay1(g.dup[x], sd, dtz);
            g.ign[x] = decay1(g.ign[x], sd, dtz);
            g.rej[x] = decay1(g.rej[x], sd, dtz);
        } else if (g.exp[x] < now) {             // delete(pg.ipStats, ip): a fresh object next time
            g.del[x] = 0.0; g.dup[x] = 0.0; g.ign[x] = 0.0; g.rej[x] = 0.0;
        }
    }
}

// AddPeer / RemovePeer (peer_gater.go:366-384) of the connections' edges
__global__ __launch_bounds__(256) void k_gater_conn(Gater g, const uint32_t* edges, int32_t n2, int32_t up,
                                                    int64_t expire)
{
    const int32_t q = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= n2) return;
    const uint32_t r = g.rep[edges[q]];
    if (up) {
        atomicAdd(&g.con[r], 1);
    } else {
        atomicSub(&g.con[r], 1);
        g.exp[r] = expire;
    }
}

// a view of a rep-indexed array in edge order (0 off the representatives)
template <typename T>
__global__ __launch_bounds__(256) void k_gater_view(const T* src, const uint32_t* rep, int64_t E, T* dst)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride)
        dst[e] = rep[e] == (uint32_t)e ? src[e] : (T)0;
}

int grid_of(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384)); }

int vfail(char* err, size_t n, const char* m)
{
    if (err && n) std::snprintf(err, n, "%s", m);
    return GSIM_EINVAL;
}

}  // namespace
}  // namespace gsim

using namespace gsim;

GaterRef gater_ref(gsim_handle* h)
{
    GaterRef r{};
    Gater* g = h->gt;
    if (!g) return r;
    r.act = g->act;
    r.gq = g->gq;
    r.del = g->del; r.dup = g->dup; r.ign = g->ign; r.rej = g->rej;
    r.a_del = g->a_del; r.a_dup = g->a_dup; r.a_ign = g->a_ign; r.a_rej = g->a_rej;
    r.a_val = g->a_val; r.a_thr = g->a_thr; r.a_last = g->a_last;
    r.tw = g->tw;
    r.dw = g->p.duplicate_weight; r.iw = g->p.ignore_weight; r.rw = g->p.reject_weight;
    r.seed = gsim_get_seed(h);
    r.n_thr = g->n_thr;
    r.direct = h->d_direct;
    r.gid = h->sh ? h->sh->d_gid : nullptr;
    return r;
}

// the gate's state for round g (before the round's delivery kernels)
int gater_round_begin(gsim_handle* h, int64_t now)
{
    Gater* g = h->gt;
    if (!g) return GSIM_OK;
    hipLaunchKernelGGL(k_gater_active, dim3(grid_of(h->n)), dim3(256), 0, h->stream, (const double*)g->val,
                       (const double*)g->thr, (const int64_t*)g->last, h->n, now, g->p.quiet_ns, g->p.threshold,
                       g->act);
    return hip_check(h, hipGetLastError(), "k_gater_active");
}

// after the commit of round `round` (its claims resolved): fold its events
int gater_fold(gsim_handle* h, int64_t round, int64_t now)
{
    Gater* g = h->gt;
    if (!g || g->fold_round != round) return GSIM_OK;
    hipLaunchKernelGGL(k_gater_fold, dim3(grid_of(std::max(h->n, h->e))), dim3(256), 0, h->stream, *g, h->n, h->e, now);
    g->fold_round = -1;
    return hip_check(h, hipGetLastError(), "k_gater_fold");
}

void gater_round_sent(gsim_handle* h, int64_t round)
{
    if (h->gt) h->gt->fold_round = round;
}

int gater_decay(gsim_handle* h, int64_t now)
{
    Gater* g = h->gt;
    if (!g) return GSIM_OK;
    hipLaunchKernelGGL(k_gater_decay, dim3(grid_of(std::max(h->n, h->e))), dim3(256), 0, h->stream, *g, h->n, h->e,
                       now);
    return hip_check(h, hipGetLastError(), "k_gater_decay");
}

int gater_connections(gsim_handle* h, const uint32_t* d_edges, int32_t n2, int32_t up, int64_t now)
{
    Gater* g = h->gt;
    if (!g || n2 <= 0) return GSIM_OK;
    hipLaunchKernelGGL(k_gater_conn, dim3((n2 + 255) / 256), dim3(256), 0, h->stream, *g, d_edges, n2, up,
                       now + g->p.retain_stats_ns);
    return hip_check(h, hipGetLastError(), "k_gater_conn");
}

void free_gater(gsim_handle* h)
{
    Gater* g = h->gt;
    if (!g) return;
    auto f = [](void* p) { if (p) (void)hipFree(p); };
    f(g->rep); f(g->gq); f(g->del); f(g->dup); f(g->ign); f(g->rej); f(g->con); f(g->exp);
    f(g->a_del); f(g->a_dup); f(g->a_ign); f(g->a_rej); f(g->val); f(g->thr); f(g->last);
    f(g->a_val); f(g->a_thr); f(g->a_last); f(g->act); f(g->tw); f(g->n_thr);
    delete g;
    h->gt = nullptr;
}

extern "C" {

int gsim_validate_peer_gater_params(const gsim_peer_gater_params* p, char* err, size_t n)
{
    // PeerGaterParams.validate (peer_gater.go:57-90), the reference's messages
    if (!p) return vfail(err, n, "nil peer gater params");
    if (p->threshold <= 0) return vfail(err, n, "invalid Threshold; must be > 0");
    if (p->global_decay <= 0 || p->global_decay >= 1) return vfail(err, n, "invalid GlobalDecay; must be between 0 and 1");
    if (p->source_decay <= 0 || p->source_decay >= 1) return vfail(err, n, "invalid SourceDecay; must be between 0 and 1");
    if (p->decay_interval_ns < 1000000000LL) return vfail(err, n, "invalid DecayInterval; must be at least 1s");
    if (p->decay_to_zero <= 0 || p->decay_to_zero >= 1) return vfail(err, n, "invalid DecayToZero; must be between 0 and 1");
    if (p->quiet_ns < 1000000000LL) return vfail(err, n, "invalud Quiet interval; must be at least 1s");
    if (p->duplicate_weight <= 0) return vfail(err, n, "invalid DuplicateWeight; must be > 0");
    if (p->ignore_weight < 1) return vfail(err, n, "invalid IgnoreWeight; must be >= 1");
    if (p->reject_weight < 1) return vfail(err, n, "invalud RejectWeight; must be >= 1");
    return GSIM_OK;
}

int gsim_default_peer_gater_params(double threshold, double global_decay, double source_decay,
                                   gsim_peer_gater_params* out)
{
    // NewPeerGaterParams (peer_gater.go:99-111) with the package defaults (:19-28)
    if (!out) return GSIM_EINVAL;
    *out = gsim_peer_gater_params{};
    out->threshold = threshold;
    out->global_decay = global_decay;
    out->source_decay = source_decay;
    out->decay_to_zero = 0.01;                          // DefaultDecayToZero (score_params.go)
    out->decay_interval_ns = 1000000000LL;              // DefaultDecayInterval
    out->retain_stats_ns = 6LL * 3600 * 1000000000LL;   // DefaultPeerGaterRetainStats
    out->quiet_ns = 60LL * 1000000000LL;                // DefaultPeerGaterQuiet
    out->duplicate_weight = 0.125;
    out->ignore_weight = 1.0;
    out->reject_weight = 16.0;
    return GSIM_OK;
}

int gsim_set_peer_gater(gsim_handle* h, const gsim_peer_gater_params* p, const double* topic_weights)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    char buf[160];
    if (gsim_validate_peer_gater_params(p, buf, sizeof buf) != GSIM_OK) { h->err = buf; return GSIM_EINVAL; }
    if (h->e == 0 || !h->dl) { h->err = "gsim_set_peer_gater needs a loaded graph and gsim_msgs_init"; return GSIM_ESTATE; }
    if (p->decay_interval_ns != h->gp.heartbeat_interval_ns) {
        h->err = "the peer gater's DecayInterval must equal the heartbeat interval (decayStats runs at every refresh)";
        return GSIM_ESTATE;
    }
    if (deliver_latency_on(h)) { h->err = "the peer gater needs messages without validation latency"; return GSIM_ESTATE; }
    const int32_t T = std::max(1, h->t);
    std::vector<unsigned long long> tw((size_t)T);
    for (int32_t t = 0; t < T; ++t) {
        double w = topic_weights ? topic_weights[t] : 0.0;
        if (w == 0) w = 1;                                          // peer_gater.go:379-381
        const double fp = w * 65536.0;
        if (!(w > 0) || fp != std::floor(fp) || fp > 4294967295.0) {
            h->err = "TopicDeliveryWeights must be positive multiples of 2^-16 below 65536";
            return GSIM_EINVAL;
        }
        tw[(size_t)t] = (unsigned long long)fp;
    }
    int rc = deliver_flush(h);
    if (rc) return rc;
    free_gater(h);
    Gater* g = new Gater();
    h->gt = g;
    g->p = *p;
    const size_t N = (size_t)h->n, E = (size_t)h->e;
    hipError_t e = hipSuccess;
    auto A = [&](void** q, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(q, std::max<size_t>(bytes, 8));
        if (e == hipSuccess) e = hipMemsetAsync(*q, 0, std::max<size_t>(bytes, 8), h->stream);
        if (e == hipSuccess) h->bytes_allocated += bytes;
    };
    A((void**)&g->rep, E * 4); A((void**)&g->gq, E * 4);
    A((void**)&g->del, E * 8); A((void**)&g->dup, E * 8); A((void**)&g->ign, E * 8); A((void**)&g->rej, E * 8);
    A((void**)&g->con, E * 4); A((void**)&g->exp, E * 8);
    A((void**)&g->a_del, E * 8); A((void**)&g->a_dup, E * 4); A((void**)&g->a_ign, E * 4); A((void**)&g->a_rej, E * 4);
    A((void**)&g->val, N * 8); A((void**)&g->thr, N * 8); A((void**)&g->last, N * 8);
    A((void**)&g->a_val, N * 4); A((void**)&g->a_thr, N * 4); A((void**)&g->a_last, N); A((void**)&g->act, N);
    A((void**)&g->tw, (size_t)T * 8); A((void**)&g->n_thr, 8);
    if (e == hipSuccess) e = hipMemcpyAsync(g->tw, tw.data(), (size_t)T * 8, hipMemcpyHostToDevice, h->stream);
    if (e != hipSuccess) { free_gater(h); return hip_check(h, e, "gsim_set_peer_gater"); }
    // on the handle's stream, after the zero fill above (a blocking copy on the
    // null stream could land first and be zeroed: lastThrottle 0, not never)
    std::vector<int64_t> never(N, kNever);
    e = hipMemcpyAsync(g->last, never.data(), N * 8, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_gater_groups, dim3(grid_of(h->e)), dim3(256), 0, h->stream, (const uint32_t*)h->d_row_ptr,
                           (const uint32_t*)h->d_col, (const uint32_t*)h->d_owner, (const uint32_t*)h->d_ip_ptr,
                           (const uint32_t*)h->d_ip_ids, (const uint8_t*)h->d_rstate, h->e, g->rep, g->con);
        hipLaunchKernelGGL(k_gater_gq, dim3(grid_of(h->e)), dim3(256), 0, h->stream, (const uint32_t*)g->rep,
                           (const uint32_t*)h->d_rev, h->e, g->gq);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) { free_gater(h); return hip_check(h, e, "gsim_set_peer_gater"); }
    return GSIM_OK;
}

int gsim_gater_throttled(gsim_handle* h, int64_t* out)
{
    if (!h || !out) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    *out = 0;
    if (!h->gt) return GSIM_OK;
    unsigned long long v = 0;
    hipError_t e = hipMemcpyAsync(&v, h->gt->n_thr, 8, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    *out = (int64_t)v;
    return hip_check(h, e, "gsim_gater_throttled");
}

int gsim_gater_read(gsim_handle* h, double* validate, double* throttle, int64_t* last, double* counters4,
                    int32_t* connected, int64_t* expire)
{
    if (!h) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    Gater* g = h->gt;
    if (!g) { h->err = "the peer gater is off (gsim_set_peer_gater)"; return GSIM_ESTATE; }
    int rc = deliver_flush(h);   // the last round's claims, then its events
    if (rc) return rc;
    const size_t N = (size_t)h->n, E = (size_t)h->e;
    hipError_t e = hipSuccess;
    auto D = [&](void* dst, const void* src, size_t bytes) {
        if (dst && e == hipSuccess) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream);
    };
    D(validate, g->val, N * 8);
    D(throttle, g->thr, N * 8);
    D(last, g->last, N * 8);
    void* tmp = nullptr;
    if (counters4 || connected || expire) e = hipMalloc(&tmp, std::max<size_t>(E * 8, 8));
    auto V = [&](const auto* src, auto* dst) {
        if (!dst || e != hipSuccess) return;
        using T = std::remove_cv_t<std::remove_pointer_t<decltype(src)>>;
        hipLaunchKernelGGL(k_gater_view<T>, dim3(grid_of(h->e)), dim3(256), 0, h->stream, src, (const uint32_t*)g->rep,
                           h->e, (T*)tmp);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(dst, tmp, E * sizeof(T), hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    };
    if (counters4) {
        V((const double*)g->del, counters4);
        V((const double*)g->dup, counters4 + E);
        V((const double*)g->ign, counters4 + 2 * E);
        V((const double*)g->rej, counters4 + 3 * E);
    }
    V((const int32_t*)g->con, connected);
    V((const int64_t*)g->exp, expire);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (tmp) (void)hipFree(tmp);
    return hip_check(h, e, "gsim_gater_read");
}

}  // extern "C"
