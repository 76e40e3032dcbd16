// TraceEventBatch encoder (include/gsim_wire.h gsim_trace_encode): the
// engine's trace records (gsim_trace_read) as the protobuf stream the
// reference's tracers write (pb/trace.proto; pubsubTracer, trace.go:70-530).
// proto2: every present field is a tag byte and a varint or a
// length-delimited body, in field-number order; sizes first, then bytes.
#include <cstring>
#include <string>

#include "gsim_wire.h"

namespace {

uint64_t vlen(uint64_t v)
{
    uint64_t n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
}

uint64_t ld(uint64_t n) { return 1 + vlen(n) + n; }

// RejectMessage reasons (tracer.go:31-38) by verdict
const char* reason_text(uint8_t v)
{
    switch (v) {
    case GSIM_VERDICT_REJECT: return "validation failed";
    case GSIM_VERDICT_IGNORE: return "validation ignored";
    case GSIM_VERDICT_THROTTLE: return "validation throttled";
    case GSIM_VERDICT_SIGNATURE: return "invalid signature";
    default: return "";
    }
}

struct Enc {
    const gsim_wire_names* names;
    const char* proto;
    uint64_t proto_len;

    uint64_t pid_len() const { return names->peer_id_len ? names->peer_id_len : 4; }
    uint64_t topic_len(int32_t t) const { return names->topic_names[t].n; }

    // the event's own message (field 4.. 16) body size, and its field number
    uint64_t body(const gsim_trace_event& e, int* field) const
    {
        const uint64_t mid = ld(8), pid = ld(pid_len());
        switch (e.type) {
        case GSIM_TRACE_PUBLISH_MESSAGE: *field = 4; return mid + ld(topic_len(e.topic));
        case GSIM_TRACE_REJECT_MESSAGE:
            *field = 5;
            return mid + pid + ld(std::strlen(reason_text(e.reason))) + ld(topic_len(e.topic));
        case GSIM_TRACE_DUPLICATE_MESSAGE: *field = 6; return mid + pid + ld(topic_len(e.topic));
        case GSIM_TRACE_DELIVER_MESSAGE: *field = 7; return mid + ld(topic_len(e.topic)) + pid;
        case GSIM_TRACE_ADD_PEER: *field = 8; return pid + ld(proto_len);
        case GSIM_TRACE_REMOVE_PEER: *field = 9; return pid;
        case GSIM_TRACE_JOIN: *field = 13; return ld(topic_len(e.topic));
        case GSIM_TRACE_LEAVE: *field = 14; return ld(topic_len(e.topic));
        case GSIM_TRACE_GRAFT: *field = 15; return pid + ld(topic_len(e.topic));
        case GSIM_TRACE_PRUNE: *field = 16; return pid + ld(topic_len(e.topic));
        default: *field = 0; return 0;
        }
    }

    uint64_t event(const gsim_trace_event& e) const
    {
        int f = 0;
        const uint64_t b = body(e, &f);
        return 1 + vlen(e.type) + ld(pid_len()) + 1 + vlen((uint64_t)e.timestamp_ns) + (f >= 16 ? 2 : 1) + vlen(b) + b;
    }

    // A message RPC (RECV_RPC / SEND_RPC) of the records [k0, k1): RPCMeta of
    // its messages, MessageMeta{messageID, topic} each (trace.go:326-345);
    // an IWANT request (reason 2): RPCMeta.control = ControlMeta{iwant =
    // [ControlIWantMeta{messageIDs}]} (trace.go:362-414), one IWANT per RPC
    // (handleIHave, gossipsub.go:692-697)
    uint64_t mmeta(const gsim_trace_event& e) const { return ld(8) + ld(topic_len(e.topic)); }
    static uint64_t iwmeta(int64_t k0, int64_t k1) { return (uint64_t)(k1 - k0) * ld(8); }
    uint64_t meta(const gsim_trace_event* ev, int64_t k0, int64_t k1) const
    {
        if (ev[k0].reason == 2) return ld(ld(iwmeta(k0, k1)));      // control { iwant { ids } }
        uint64_t s = 0;
        for (int64_t k = k0; k < k1; ++k) s += ld(mmeta(ev[k]));
        return s;
    }
    uint64_t rpc_body(const gsim_trace_event* ev, int64_t k0, int64_t k1) const
    {
        return ld(pid_len()) + ld(meta(ev, k0, k1));             // receivedFrom / sendTo, meta
    }
    uint64_t rpc_event(const gsim_trace_event* ev, int64_t k0, int64_t k1) const
    {
        const gsim_trace_event& e = ev[k0];
        const uint64_t b = rpc_body(ev, k0, k1);
        return 1 + vlen(e.type) + ld(pid_len()) + 1 + vlen((uint64_t)e.timestamp_ns) + 1 + vlen(b) + b;
    }
};

bool is_rpc(const gsim_trace_event& e) { return e.type == GSIM_TRACE_RECV_RPC || e.type == GSIM_TRACE_SEND_RPC; }

// the records one TraceEvent covers: [k, end) -- an IWANT answer's messages
// (reason 1) or an IWANT request's ids (reason 2) to one peer in one round
// are one RPC, everything else one record
int64_t unit_end(const gsim_trace_event* ev, int64_t n, int64_t k)
{
    int64_t q = k + 1;
    if (is_rpc(ev[k]) && (ev[k].reason == 1 || ev[k].reason == 2))
        while (q < n && ev[q].type == ev[k].type && ev[q].reason == ev[k].reason &&
               ev[q].timestamp_ns == ev[k].timestamp_ns &&
               ev[q].peer == ev[k].peer && ev[q].other == ev[k].other)
            ++q;
    return q;
}

struct W {
    uint8_t* p;
    void byte(uint8_t b) { *p++ = b; }
    void varint(uint64_t v)
    {
        while (v >= 0x80) { *p++ = (uint8_t)(v | 0x80); v >>= 7; }
        *p++ = (uint8_t)v;
    }
    void tag(int field, int wt)
    {
        varint((uint64_t)((field << 3) | wt));
    }
    void raw(int field, const void* s, uint64_t n)
    {
        tag(field, 2);
        varint(n);
        if (n) std::memcpy(p, s, n);
        p += n;
    }
};

void put_peer(W& w, const Enc& c, int field, uint32_t peer)
{
    if (c.names->peer_id_len) {
        w.raw(field, c.names->peer_ids + (size_t)peer * c.names->peer_id_len, c.names->peer_id_len);
    } else {
        const uint8_t b[4] = {(uint8_t)(peer >> 24), (uint8_t)(peer >> 16), (uint8_t)(peer >> 8), (uint8_t)peer};
        w.raw(field, b, 4);
    }
}

void put_mid(W& w, int field, uint64_t id)
{
    uint8_t b[8];
    for (int s = 0; s < 8; ++s) b[s] = (uint8_t)(id >> (56 - 8 * s));
    w.raw(field, b, 8);
}

void put_topic(W& w, const Enc& c, int field, int32_t t)
{
    w.raw(field, c.names->topic_names[t].p, c.names->topic_names[t].n);
}

}  // namespace

extern "C" int gsim_trace_encode(const gsim_trace_event* ev, int64_t n, const gsim_wire_names* names,
                                 const char* proto, uint8_t* out, uint64_t cap, uint64_t* len)
{
    if (!len || n < 0 || (n > 0 && (!ev || !names || !names->topic_names))) return GSIM_EINVAL;
    if (names && names->peer_id_len && !names->peer_ids) return GSIM_EINVAL;
    Enc c{names, proto ? proto : "", proto ? std::strlen(proto) : 0};
    uint64_t total = 0;
    for (int64_t k = 0; k < n;) {
        const int64_t k1 = unit_end(ev, n, k);
        int f = 0;
        (void)c.body(ev[k], &f);
        if (!f && !is_rpc(ev[k])) return GSIM_EINVAL;
        for (int64_t q = k; q < k1; ++q)
            if (ev[q].topic < 0 && is_rpc(ev[q])) return GSIM_EINVAL;
        total += ld(is_rpc(ev[k]) ? c.rpc_event(ev, k, k1) : c.event(ev[k]));   // TraceEventBatch.batch = 1
        k = k1;
    }
    *len = total;
    if (total > cap || (total && !out)) return GSIM_ERANGE;
    W w{out};
    for (int64_t k = 0; k < n;) {
        const int64_t k1 = unit_end(ev, n, k);
        const gsim_trace_event& e = ev[k];
        if (is_rpc(e)) {
            w.tag(1, 2);
            w.varint(c.rpc_event(ev, k, k1));
            w.tag(1, 0);                                     // type
            w.varint(e.type);
            put_peer(w, c, 2, e.peer);                       // peerID
            w.tag(3, 0);                                     // timestamp
            w.varint((uint64_t)e.timestamp_ns);
            w.tag(e.type == GSIM_TRACE_RECV_RPC ? 10 : 11, 2);   // recvRPC = 10 / sendRPC = 11
            w.varint(c.rpc_body(ev, k, k1));
            put_peer(w, c, 1, e.other);                      // receivedFrom / sendTo
            w.tag(2, 2);                                     // meta
            w.varint(c.meta(ev, k, k1));
            if (e.reason == 2) {                             // RPCMeta.control = 3 { iwant = 2 { messageIDs = 1 } }
                const uint64_t iw = Enc::iwmeta(k, k1);
                w.tag(3, 2);
                w.varint(ld(iw));
                w.tag(2, 2);
                w.varint(iw);
                for (int64_t q = k; q < k1; ++q) put_mid(w, 1, ev[q].msg_id);
                k = k1;
                continue;
            }
            for (int64_t q = k; q < k1; ++q) {               // RPCMeta.messages = 1
                w.tag(1, 2);
                w.varint(c.mmeta(ev[q]));
                put_mid(w, 1, ev[q].msg_id);
                put_topic(w, c, 2, ev[q].topic);
            }
            k = k1;
            continue;
        }
        k = k1;
        w.tag(1, 2);
        w.varint(c.event(e));
        w.tag(1, 0);                                         // type
        w.varint(e.type);
        put_peer(w, c, 2, e.peer);                           // peerID
        w.tag(3, 0);                                         // timestamp
        w.varint((uint64_t)e.timestamp_ns);
        int f = 0;
        const uint64_t b = c.body(e, &f);
        w.tag(f, 2);
        w.varint(b);
        switch (e.type) {
        case GSIM_TRACE_PUBLISH_MESSAGE:                     // messageID, topic
            put_mid(w, 1, e.msg_id);
            put_topic(w, c, 2, e.topic);
            break;
        case GSIM_TRACE_REJECT_MESSAGE: {                    // messageID, receivedFrom, reason, topic
            put_mid(w, 1, e.msg_id);
            put_peer(w, c, 2, e.other);
            const char* r = reason_text(e.reason);
            w.raw(3, r, std::strlen(r));
            put_topic(w, c, 4, e.topic);
            break;
        }
        case GSIM_TRACE_DUPLICATE_MESSAGE:                   // messageID, receivedFrom, topic
            put_mid(w, 1, e.msg_id);
            put_peer(w, c, 2, e.other);
            put_topic(w, c, 3, e.topic);
            break;
        case GSIM_TRACE_DELIVER_MESSAGE:                     // messageID, topic, receivedFrom
            put_mid(w, 1, e.msg_id);
            put_topic(w, c, 2, e.topic);
            put_peer(w, c, 3, e.other);
            break;
        case GSIM_TRACE_ADD_PEER:                            // peerID, proto
            put_peer(w, c, 1, e.other);
            w.raw(2, c.proto, c.proto_len);
            break;
        case GSIM_TRACE_REMOVE_PEER:                         // peerID
            put_peer(w, c, 1, e.other);
            break;
        case GSIM_TRACE_JOIN:                                // topic = 1
            put_topic(w, c, 1, e.topic);
            break;
        case GSIM_TRACE_LEAVE:                               // topic = 2 (pb/trace.proto:92-94)
            put_topic(w, c, 2, e.topic);
            break;
        default:                                             // GRAFT / PRUNE: peerID, topic
            put_peer(w, c, 1, e.other);
            put_topic(w, c, 2, e.topic);
            break;
        }
    }
    return GSIM_OK;
}

// ---- SendRPC / RecvRPC / DropRPC (trace.go:250-324) ----------------------
// The RPCMeta of an encoded RPC as traceRPCMeta builds it (trace.go:326-414):
// messages -> MessageMeta{messageID = from || seqno (DefaultMsgIdFn),
// topic}; subscriptions -> SubMeta{subscribe, topic}; control (present
// whenever the RPC has one) -> ControlMeta{ihave{topic, messageIDs},
// iwant{messageIDs}, graft{topic}, prune{topic, peers = PeerInfo.peerID}}.
// Optional fields are copied when present in the RPC, as the Go pointers
// are; repeated bytes elements always (an absent peerID is an empty one).
namespace {

struct Rd {
    const uint8_t* p;
    const uint8_t* e;
    bool ok = true;
    bool more() const { return ok && p < e; }
    uint64_t varint()
    {
        uint64_t v = 0;
        for (int s = 0; s < 64 && p < e; s += 7) {
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << s;
            if (!(b & 0x80)) return v;
        }
        ok = false;
        return 0;
    }
    // the next field: number, wire type; length-delimited payload in (q, n)
    bool field(int* f, int* wt, const uint8_t** q, uint64_t* n, uint64_t* v)
    {
        const uint64_t k = varint();
        if (!ok) return false;
        *f = (int)(k >> 3);
        *wt = (int)(k & 7);
        *q = nullptr; *n = 0; *v = 0;
        switch (*wt) {
        case 0: *v = varint(); break;
        case 1: if (e - p < 8) ok = false; else p += 8; break;
        case 5: if (e - p < 4) ok = false; else p += 4; break;
        case 2: {
            const uint64_t L = varint();
            if (!ok || (uint64_t)(e - p) < L) { ok = false; break; }
            *q = p; *n = L; p += L;
            break;
        }
        default: ok = false;
        }
        return ok;
    }
};

struct Pw {
    std::string s;
    void varint(uint64_t v)
    {
        while (v >= 0x80) { s.push_back((char)(v | 0x80)); v >>= 7; }
        s.push_back((char)v);
    }
    void tag(int f, int wt) { varint((uint64_t)((f << 3) | wt)); }
    void bytes(int f, const void* q, uint64_t n)
    {
        tag(f, 2);
        varint(n);
        s.append((const char*)q, (size_t)n);
    }
    void sub(int f, const std::string& body) { bytes(f, body.data(), body.size()); }
    void u64(int f, uint64_t v) { tag(f, 0); varint(v); }
};

// copy the length-delimited fields `from` -> `to` of a message (optional
// ones present / repeated ones in order), everything else dropped
bool remap(const uint8_t* q, uint64_t n, const int* from, const int* to, int k, Pw* w)
{
    Rd r{q, q + n};
    int f, wt;
    const uint8_t* b;
    uint64_t L, v;
    // fields in ascending output order: one pass per output field
    for (int x = 0; x < k; ++x) {
        r = Rd{q, q + n};
        while (r.more()) {
            if (!r.field(&f, &wt, &b, &L, &v)) return false;
            if (f == from[x] && wt == 2) w->bytes(to[x], b, L);
        }
    }
    return r.ok;
}

bool rpc_meta(const uint8_t* q, uint64_t n, Pw* meta)
{
    Rd r{q, q + n};
    int f, wt;
    const uint8_t* b;
    uint64_t L, v;
    // messages (RPC.publish = 2) -> RPCMeta.messages = 1
    while (r.more()) {
        if (!r.field(&f, &wt, &b, &L, &v)) return false;
        if (f != 2 || wt != 2) continue;
        Rd m{b, b + L};
        std::string from, seqno;
        const uint8_t* tp = nullptr;
        uint64_t tn = 0;
        bool has_topic = false;
        int mf, mwt;
        const uint8_t* mb;
        uint64_t ml, mv;
        while (m.more()) {
            if (!m.field(&mf, &mwt, &mb, &ml, &mv)) return false;
            if (mwt != 2) continue;
            if (mf == 1) from.assign((const char*)mb, ml);
            else if (mf == 3) seqno.assign((const char*)mb, ml);
            else if (mf == 4) { tp = mb; tn = ml; has_topic = true; }
        }
        Pw mm;
        const std::string id = from + seqno;
        mm.bytes(1, id.data(), id.size());
        if (has_topic) mm.bytes(2, tp, tn);
        meta->sub(1, mm.s);
    }
    if (!r.ok) return false;
    // subscriptions (1) -> subscription = 2: SubOpts{subscribe = 1, topicid = 2}
    r = Rd{q, q + n};
    while (r.more()) {
        if (!r.field(&f, &wt, &b, &L, &v)) return false;
        if (f != 1 || wt != 2) continue;
        Rd m{b, b + L};
        Pw sm;
        bool has_sub = false, subv = false, has_topic = false;
        const uint8_t* tp = nullptr;
        uint64_t tn = 0;
        int mf, mwt;
        const uint8_t* mb;
        uint64_t ml, mv;
        while (m.more()) {
            if (!m.field(&mf, &mwt, &mb, &ml, &mv)) return false;
            if (mf == 1 && mwt == 0) { has_sub = true; subv = mv != 0; }
            else if (mf == 2 && mwt == 2) { has_topic = true; tp = mb; tn = ml; }
        }
        if (has_sub) sm.u64(1, subv ? 1 : 0);
        if (has_topic) sm.bytes(2, tp, tn);
        meta->sub(2, sm.s);
    }
    if (!r.ok) return false;
    // control (3) -> control = 3 (the last one, as proto2 merges; one in practice)
    r = Rd{q, q + n};
    bool has_ctl = false;
    Pw cm;
    while (r.more()) {
        if (!r.field(&f, &wt, &b, &L, &v)) return false;
        if (f != 3 || wt != 2) continue;
        has_ctl = true;
        cm.s.clear();
        static const int ih_from[] = {1, 2}, ih_to[] = {1, 2};     // ControlIHave{topicID, messageIDs}
        static const int iw_from[] = {1}, iw_to[] = {1};            // ControlIWant{messageIDs}
        static const int gr_from[] = {1}, gr_to[] = {1};            // ControlGraft{topicID}
        for (int kind = 1; kind <= 4; ++kind) {
            Rd c{b, b + L};
            int cf, cwt;
            const uint8_t* cb;
            uint64_t cl, cv;
            while (c.more()) {
                if (!c.field(&cf, &cwt, &cb, &cl, &cv)) return false;
                if (cf != kind || cwt != 2) continue;
                Pw x;
                bool ok = true;
                if (kind == 1) ok = remap(cb, cl, ih_from, ih_to, 2, &x);
                else if (kind == 2) ok = remap(cb, cl, iw_from, iw_to, 1, &x);
                else if (kind == 3) ok = remap(cb, cl, gr_from, gr_to, 1, &x);
                else {
                    // ControlPrune{topicID = 1, peers = 2 (PeerInfo{peerID = 1})}
                    ok = remap(cb, cl, gr_from, gr_to, 1, &x);
                    Rd pr{cb, cb + cl};
                    int pf, pwt;
                    const uint8_t* pb;
                    uint64_t pl, pv;
                    while (ok && pr.more()) {
                        if (!pr.field(&pf, &pwt, &pb, &pl, &pv)) return false;
                        if (pf != 2 || pwt != 2) continue;
                        Rd pi{pb, pb + pl};
                        const uint8_t* id = nullptr;
                        uint64_t idn = 0;
                        int qf, qwt;
                        const uint8_t* qb;
                        uint64_t ql, qv;
                        while (pi.more()) {
                            if (!pi.field(&qf, &qwt, &qb, &ql, &qv)) return false;
                            if (qf == 1 && qwt == 2) { id = qb; idn = ql; }
                        }
                        x.bytes(2, id, idn);
                    }
                }
                if (!ok) return false;
                cm.sub(kind, x.s);
            }
            if (!c.ok) return false;
        }
    }
    if (!r.ok) return false;
    if (has_ctl) meta->sub(3, cm.s);
    return true;
}

}  // namespace

extern "C" int gsim_trace_rpc_encode(const uint8_t* rpcs, const gsim_wire_ref* refs, int64_t n,
                                     const gsim_wire_names* names, int64_t timestamp_ns, int32_t which, uint8_t* out,
                                     uint64_t cap, uint64_t* len)
{
    if (!len || n < 0 || (n > 0 && (!rpcs || !refs || !names)) || (which & ~7) || !which) return GSIM_EINVAL;
    if (names && names->peer_id_len && !names->peer_ids) return GSIM_EINVAL;
    auto pid = [&](uint32_t p) -> std::string {
        if (names->peer_id_len)
            return std::string((const char*)names->peer_ids + (size_t)p * names->peer_id_len, names->peer_id_len);
        const char b[4] = {(char)(p >> 24), (char)(p >> 16), (char)(p >> 8), (char)p};
        return std::string(b, 4);
    };
    Pw batch;
    for (int64_t k = 0; k < n; ++k) {
        const gsim_wire_ref& r = refs[k];
        Pw meta;
        if (!rpc_meta(rpcs + r.offset, r.len, &meta)) return GSIM_EINVAL;
        // SEND_RPC = 7 (sendRPC = 11), RECV_RPC = 6 (recvRPC = 10), DROP_RPC = 8 (dropRPC = 12)
        static const int kType[3] = {7, 6, 8}, kField[3] = {11, 10, 12};
        for (int q = 0; q < 3; ++q) {
            if (!((which >> q) & 1)) continue;
            const bool recv = q == 1;
            Pw body;
            const std::string other = pid(recv ? r.from : r.to);   // receivedFrom / sendTo
            body.bytes(1, other.data(), other.size());
            body.sub(2, meta.s);
            Pw ev;
            ev.u64(1, (uint64_t)kType[q]);
            const std::string me = pid(recv ? r.to : r.from);
            ev.bytes(2, me.data(), me.size());
            ev.u64(3, (uint64_t)timestamp_ns);
            ev.sub(kField[q], body.s);
            batch.sub(1, ev.s);
        }
    }
    *len = batch.s.size();
    if (batch.s.size() > cap || (!batch.s.empty() && !out)) return GSIM_ERANGE;
    if (!batch.s.empty()) std::memcpy(out, batch.s.data(), batch.s.size());
    return GSIM_OK;
}

// PBTracer's file (tracer.go:130-179): protoio.NewDelimitedWriter writes each
// TraceEvent as its uvarint length then its bytes.  A TraceEventBatch holds the
// same events as field 1 entries (tag 0x0a, length, bytes): dropping each tag
// gives the delimited stream.
extern "C" int gsim_trace_delimited(const uint8_t* batch, uint64_t len, uint8_t* out, uint64_t cap, uint64_t* n)
{
    if (!n || (len && !batch)) return GSIM_EINVAL;
    Rd r{batch, batch + len};
    uint64_t total = 0;
    int f, wt;
    const uint8_t* q;
    uint64_t L, v;
    while (r.more()) {
        if (!r.field(&f, &wt, &q, &L, &v) || f != 1 || wt != 2) return GSIM_EINVAL;
        total += vlen(L) + L;
    }
    if (!r.ok) return GSIM_EINVAL;
    *n = total;
    if (total > cap || (total && !out)) return GSIM_ERANGE;
    W w{out};
    r = Rd{batch, batch + len};
    while (r.more()) {
        r.field(&f, &wt, &q, &L, &v);
        w.varint(L);
        if (L) std::memcpy(w.p, q, L);
        w.p += L;
    }
    return GSIM_OK;
}

