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
};

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
    for (int64_t k = 0; k < n; ++k) {
        int f = 0;
        (void)c.body(ev[k], &f);
        if (!f) return GSIM_EINVAL;
        total += ld(c.event(ev[k]));                        // TraceEventBatch.batch = 1
    }
    *len = total;
    if (total > cap || (total && !out)) return GSIM_ERANGE;
    W w{out};
    for (int64_t k = 0; k < n; ++k) {
        const gsim_trace_event& e = ev[k];
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
