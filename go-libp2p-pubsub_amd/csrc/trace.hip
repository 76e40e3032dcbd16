// Trace export (include/gsim.h gsim_trace_config / gsim_trace_read;
// SURVEY.md §8(f) row 2): the events pubsubTracer hands to a TraceEvent sink
// (trace.go:70-530, pb/trace.proto) for a range of routers.
//
// The kernels append events as they happen (gsim_internal.h TraceRef): the
// origin's publication (k_publish), every message copy that passes AcceptFrom
// (k_send_tm / k_send / k_gossip_deliver), the router's mesh additions and
// removals (the heartbeat's graftPeer / prunePeer, handleGraft,
// handlePrune) and connection churn (k_churn_apply).  Whether a copy was the
// first reception is decided only when every copy of its round has claimed
// (the lowest receiving edge wins), so a copy is recorded unclassified and
// k_trace_resolve settles it at read time from the receiver's seen-set cell
// (first-seen round + first sender): the first reception of an accepted
// message is DELIVER_MESSAGE, of a rejected / ignored / throttled one
// REJECT_MESSAGE with the verdict as its reason (pushMsg -> validate,
// pubsub.go:1118-1162, validation.go:282-345), any other copy
// DUPLICATE_MESSAGE.  Bad-signature copies are rejected before markSeen and
// recorded as REJECT_MESSAGE directly.
#include <algorithm>
#include <tuple>
#include <vector>

#include "gsim_internal.h"

namespace gsim {
namespace {

// events [k0, n): those before k0 were resolved by an earlier read (TraceRef::resolved)
__global__ __launch_bounds__(256) void k_trace_resolve(gsim_trace_event* ev, int64_t k0, int64_t n, TraceView v)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = k0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        gsim_trace_event x = ev[k];
        if (x.type == GSIM_TRACE_SEND_RPC || x.type == GSIM_TRACE_RECV_RPC) {   // round << 32 | slot: the id
            ev[k].msg_id = v.mid[(uint32_t)x.msg_id];
            continue;
        }
        if (x.type != kTraceCopy) continue;
        const uint32_t m = (uint32_t)x.msg_id;
        const int64_t g = (int64_t)(x.msg_id >> 32);
        const uint64_t c = v.cells.get(m, (int32_t)v.mtopic[m], x.peer);
        // every claim is committed before a read (gsim_trace_read flushes)
        const int64_t fr = c == kUnseen64 ? -1 : (int64_t)(c >> 32);
        const uint32_t from = (uint32_t)c & kPeerMask;
        const uint8_t vd = v.minv[m];
        // a validation latency L: seen in round fr - L, verdict traced when
        // validation completes in round fr (validation.go:334-341)
        const int64_t L = v.mlat ? v.mlat[m] : 0;
        if (fr >= 0 && fr - L == g && from == x.other) {
            x.type = vd == GSIM_VERDICT_ACCEPT ? GSIM_TRACE_DELIVER_MESSAGE : GSIM_TRACE_REJECT_MESSAGE;
            x.reason = vd == GSIM_VERDICT_ACCEPT ? 0 : vd;
            if (L) {
                const int64_t q = fr / v.rounds;
                x.timestamp_ns = v.t0 + q * v.hb + v.roff[fr - q * v.rounds];
            }
        } else {
            x.type = GSIM_TRACE_DUPLICATE_MESSAGE;
            x.reason = 0;
        }
        x.msg_id = v.mid[m];
        ev[k] = x;
    }
}

// bad-signature copies carry round << 32 | slot too: only the id changes
__global__ __launch_bounds__(256) void k_trace_sig_ids(gsim_trace_event* ev, int64_t k0, int64_t n, const uint64_t* mid)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = k0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        gsim_trace_event x = ev[k];
        if (x.type != GSIM_TRACE_REJECT_MESSAGE || x.reason != GSIM_VERDICT_SIGNATURE) continue;
        ev[k].msg_id = mid[(uint32_t)x.msg_id];
    }
}

void trace_free(gsim_handle* h)
{
    if (h->trace.ev) (void)hipFree(h->trace.ev);
    if (h->trace.n) (void)hipFree(h->trace.n);
    h->trace = TraceRef{};
}

}  // namespace
}  // namespace gsim

using namespace gsim;

extern "C" {

int gsim_trace_config(gsim_handle* h, uint32_t peer_lo, uint32_t peer_hi, int64_t cap)
{
    if (!h) return GSIM_EINVAL;
    if (h->sh) { h->err = "a shard traces through gsim_group_trace_config (global ids)"; return GSIM_ESTATE; }
    return trace_config_local(h, peer_lo, peer_hi, peer_lo, peer_hi, cap);
}

}  // extern "C"

// Trace the local routers [lo, hi) (owned) and accept events of [xlo, xhi)
// (owned and ghosts) where only this engine knows of them (TraceRef::on_any).
int trace_config_local(gsim_handle* h, uint32_t peer_lo, uint32_t peer_hi, uint32_t xlo, uint32_t xhi, int64_t cap)
{
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    if (cap < 0 || peer_lo > peer_hi || (int64_t)peer_hi > h->n || xlo > xhi || (int64_t)xhi > h->n) return GSIM_EINVAL;
    (void)hipStreamSynchronize(h->stream);
    trace_free(h);
    if (cap == 0) return GSIM_OK;
    TraceRef t;
    hipError_t e = hipMalloc((void**)&t.ev, sizeof(gsim_trace_event) * (size_t)cap);
    if (e == hipSuccess) e = hipMalloc((void**)&t.n, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(t.n, 0, sizeof(uint32_t), h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        if (t.ev) (void)hipFree(t.ev);
        if (t.n) (void)hipFree(t.n);
        return hip_check(h, e, "gsim_trace_config");
    }
    t.cap = std::min<int64_t>(cap, 0xFFFFFFFFll);
    t.lo = peer_lo;
    t.hi = peer_hi;
    t.xlo = xlo;
    t.xhi = xhi;
    h->trace = t;
    return GSIM_OK;
}

extern "C" {

int gsim_trace_read(gsim_handle* h, gsim_trace_event* out, int64_t cap, int64_t* n)
{
    if (!h || !n) return GSIM_EINVAL;
    if (hipSetDevice(h->device) != hipSuccess) return GSIM_EDEVICE;
    *n = 0;
    if (!h->trace.ev) { h->err = "tracing is off (gsim_trace_config)"; return GSIM_ESTATE; }
    int rc = deliver_flush(h);                     // the last round's claims decide its first receptions
    if (rc) return rc;
    uint32_t cnt = 0;
    hipError_t e = hipMemcpyAsync(&cnt, h->trace.n, sizeof(cnt), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "trace count");
    if ((int64_t)cnt > h->trace.cap) {
        h->err = "the trace buffer overflowed (raise the gsim_trace_config capacity)";
        return GSIM_ERANGE;
    }
    *n = cnt;
    if (!out) return GSIM_OK;                      // a query: nothing consumed
    if ((int64_t)cnt > cap) { h->err = "output buffer too small for the traced events"; return GSIM_ERANGE; }
    if (cnt) {
        TraceView v{};
        const bool have = deliver_trace_view(h, &v);
        // the events an earlier read kept are resolved already
        const int64_t k0 = std::min<int64_t>(h->trace.resolved, cnt);
        const int grid = (int)std::min<int64_t>(((int64_t)cnt - k0 + 255) / 256, 4096);
        if (have && grid > 0) {
            hipLaunchKernelGGL(k_trace_resolve, dim3(grid), dim3(256), 0, h->stream, h->trace.ev, k0, (int64_t)cnt, v);
            hipLaunchKernelGGL(k_trace_sig_ids, dim3(grid), dim3(256), 0, h->stream, h->trace.ev, k0, (int64_t)cnt,
                               v.mid);
            e = hipGetLastError();
        }
        if (e == hipSuccess)
            e = hipMemcpyAsync(out, h->trace.ev, sizeof(gsim_trace_event) * cnt, hipMemcpyDeviceToHost, h->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_trace_read");
    // a first reception whose validation completes after the last round run
    // (gsim_msg.vdelay) is traced when it completes: its resolved event stays
    // in the buffer for a later read
    const int64_t tlast = deliver_last_round_time(h);
    gsim_trace_event* mid = std::stable_partition(out, out + cnt,
                                                  [tlast](const gsim_trace_event& x) { return x.timestamp_ns <= tlast; });
    const uint32_t keep = (uint32_t)(out + cnt - mid);
    if (keep) e = hipMemcpyAsync(h->trace.ev, mid, sizeof(gsim_trace_event) * keep, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h->trace.n, &keep, sizeof(uint32_t), hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_check(h, e, "gsim_trace_read");
    h->trace.resolved = keep;                      // the kept events lead the buffer, resolved
    cnt -= keep;
    *n = cnt;
    std::sort(out, out + cnt, [](const gsim_trace_event& a, const gsim_trace_event& b) {
        // (reason before topic: one IWANT answer's messages stay together, gsim_trace_encode)
        return std::tie(a.timestamp_ns, a.peer, a.type, a.other, a.reason, a.topic, a.msg_id) <
               std::tie(b.timestamp_ns, b.peer, b.type, b.other, b.reason, b.topic, b.msg_id);
    });
    return GSIM_OK;
}

}  // extern "C"

void trace_release(gsim_handle* h) { gsim::trace_free(h); }
