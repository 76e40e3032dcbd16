// Host encoders of the GossipSub wire format (include/gsim_wire.h).
//
// The RPC messages of pb/rpc.proto:5-57 are proto2: every field is a tag
// byte (field number << 3 | wire type) followed by a varint or a
// length-delimited body, in field-number order (gogo-protobuf's generated
// Marshal writes the fields back to front into a sized buffer, which leaves
// them in ascending order; rpc.pb.go MarshalToSizedBuffer).  Sizes are
// computed first (Size()), then the bytes are written front to back.
//
// fragmentRPC (gossipsub.go:1204-1296) and fragmentMessageIds (1298-1318)
// are restated on index lists into the input tables, so a fragment costs no
// copies of message bodies until it is encoded.
#include <cstring>
#include <string>
#include <vector>

#include "gsim_wire.h"

namespace {

uint64_t varint_len(uint64_t v)
{
    uint64_t n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
}

// a length-delimited field with a body of n bytes: tag + length + body
uint64_t ld(uint64_t n) { return 1 + varint_len(n) + n; }
uint64_t opt_bytes(const gsim_bytes& b) { return b.p ? ld(b.n) : 0; }

struct Writer {
    uint8_t* p;
    void byte(uint8_t b) { *p++ = b; }
    void varint(uint64_t v)
    {
        while (v >= 0x80) { *p++ = (uint8_t)(v | 0x80); v >>= 7; }
        *p++ = (uint8_t)v;
    }
    void bytes(uint8_t tag, const gsim_bytes& b)
    {
        if (!b.p) return;
        byte(tag);
        varint(b.n);
        if (b.n) std::memcpy(p, b.p, b.n);
        p += b.n;
    }
};

// ---- message sizes (the bodies, as Go's Size()) ----------------------------

uint64_t sub_size(const gsim_wire_sub& s)
{
    return (s.subscribe >= 0 ? 2 : 0) + opt_bytes(s.topic);
}

uint64_t msg_size(const gsim_wire_msg& m)
{
    return opt_bytes(m.from) + opt_bytes(m.data) + opt_bytes(m.seqno) + opt_bytes(m.topic) +
           opt_bytes(m.signature) + opt_bytes(m.key);
}

uint64_t ids_size(const gsim_wire_rpc& r, const uint32_t* idx, uint32_t n)
{
    uint64_t s = 0;
    for (uint32_t k = 0; k < n; ++k) s += ld(r.ids[idx[k]].n);
    return s;
}

uint64_t px_size(const gsim_wire_px& x) { return opt_bytes(x.peer) + opt_bytes(x.record); }

uint64_t prune_size(const gsim_wire_rpc& r, const gsim_wire_prune& pr)
{
    uint64_t s = opt_bytes(pr.topic);
    for (uint32_t k = 0; k < pr.npx; ++k) s += ld(px_size(r.px[pr.px0 + k]));
    if (pr.has_backoff) s += 1 + varint_len(pr.backoff);
    return s;
}

uint64_t graft_size(const gsim_wire_graft& g) { return opt_bytes(g.topic); }

// An RPC as lists of indices into the input tables (a fragment, or the input
// itself).  IHAVE / IWANT items carry their own id lists; a fragmented IHAVE
// has no topic (gossipsub.go:1288).
struct Gossip {
    bool has_topic;
    gsim_bytes topic;
    std::vector<uint32_t> ids;
};

struct Frag {
    std::vector<uint32_t> subs, msgs, graft, prune;
    std::vector<Gossip> ihave, iwant;
    bool has_control = false;
};

uint64_t gossip_size(const gsim_wire_rpc& r, const Gossip& g)
{
    return (g.has_topic ? opt_bytes(g.topic) : 0) + ids_size(r, g.ids.data(), (uint32_t)g.ids.size());
}

uint64_t control_size(const gsim_wire_rpc& r, const Frag& f)
{
    uint64_t s = 0;
    for (const auto& g : f.ihave) s += ld(gossip_size(r, g));
    for (const auto& g : f.iwant) s += ld(gossip_size(r, g));
    for (uint32_t k : f.graft) s += ld(graft_size(r.graft[k]));
    for (uint32_t k : f.prune) s += ld(prune_size(r, r.prune[k]));
    return s;
}

uint64_t frag_size(const gsim_wire_rpc& r, const Frag& f)
{
    uint64_t s = 0;
    for (uint32_t k : f.subs) s += ld(sub_size(r.subs[k]));
    for (uint32_t k : f.msgs) s += ld(msg_size(r.msgs[k]));
    if (f.has_control) s += ld(control_size(r, f));
    return s;
}

void write_gossip(Writer& w, const gsim_wire_rpc& r, const Gossip& g, uint8_t id_tag)
{
    if (g.has_topic) w.bytes(0x0a, g.topic);
    for (uint32_t k : g.ids) w.bytes(id_tag, r.ids[k]);
}

void write_frag(Writer& w, const gsim_wire_rpc& r, const Frag& f)
{
    for (uint32_t k : f.subs) {                            // RPC.subscriptions = 1
        const gsim_wire_sub& s = r.subs[k];
        w.byte(0x0a);
        w.varint(sub_size(s));
        if (s.subscribe >= 0) { w.byte(0x08); w.byte(s.subscribe ? 1 : 0); }
        w.bytes(0x12, s.topic);
    }
    for (uint32_t k : f.msgs) {                            // RPC.publish = 2
        const gsim_wire_msg& m = r.msgs[k];
        w.byte(0x12);
        w.varint(msg_size(m));
        w.bytes(0x0a, m.from);
        w.bytes(0x12, m.data);
        w.bytes(0x1a, m.seqno);
        w.bytes(0x22, m.topic);
        w.bytes(0x2a, m.signature);
        w.bytes(0x32, m.key);
    }
    if (!f.has_control) return;
    w.byte(0x1a);                                          // RPC.control = 3
    w.varint(control_size(r, f));
    for (const auto& g : f.ihave) {                        // ControlMessage.ihave = 1
        w.byte(0x0a);
        w.varint(gossip_size(r, g));
        write_gossip(w, r, g, 0x12);                       // ControlIHave.messageIDs = 2
    }
    for (const auto& g : f.iwant) {                        // ControlMessage.iwant = 2
        w.byte(0x12);
        w.varint(gossip_size(r, g));
        write_gossip(w, r, g, 0x0a);                       // ControlIWant.messageIDs = 1
    }
    for (uint32_t k : f.graft) {                           // ControlMessage.graft = 3
        w.byte(0x1a);
        w.varint(graft_size(r.graft[k]));
        w.bytes(0x0a, r.graft[k].topic);
    }
    for (uint32_t k : f.prune) {                           // ControlMessage.prune = 4
        const gsim_wire_prune& pr = r.prune[k];
        w.byte(0x22);
        w.varint(prune_size(r, pr));
        w.bytes(0x0a, pr.topic);
        for (uint32_t q = 0; q < pr.npx; ++q) {            // ControlPrune.peers = 2
            const gsim_wire_px& x = r.px[pr.px0 + q];
            w.byte(0x12);
            w.varint(px_size(x));
            w.bytes(0x0a, x.peer);
            w.bytes(0x12, x.record);
        }
        if (pr.has_backoff) { w.byte(0x18); w.varint(pr.backoff); }   // ControlPrune.backoff = 3
    }
}

Frag whole(const gsim_wire_rpc& r)
{
    Frag f;
    for (uint32_t k = 0; k < r.nsubs; ++k) f.subs.push_back(k);
    for (uint32_t k = 0; k < r.nmsgs; ++k) f.msgs.push_back(k);
    f.has_control = r.has_control != 0;
    if (!f.has_control) return f;
    for (uint32_t k = 0; k < r.nihave; ++k) {
        Gossip g{r.ihave[k].topic.p != nullptr, r.ihave[k].topic, {}};
        for (uint32_t q = 0; q < r.ihave[k].nid; ++q) g.ids.push_back(r.ihave[k].id0 + q);
        f.ihave.push_back(std::move(g));
    }
    for (uint32_t k = 0; k < r.niwant; ++k) {
        Gossip g{false, {nullptr, 0}, {}};
        for (uint32_t q = 0; q < r.iwant[k].nid; ++q) g.ids.push_back(r.iwant[k].id0 + q);
        f.iwant.push_back(std::move(g));
    }
    for (uint32_t k = 0; k < r.ngraft; ++k) f.graft.push_back(k);
    for (uint32_t k = 0; k < r.nprune; ++k) f.prune.push_back(k);
    return f;
}

bool tables_ok(const gsim_wire_rpc* r)
{
    if (!r) return false;
    if ((r->nsubs && !r->subs) || (r->nmsgs && !r->msgs) || (r->nihave && !r->ihave) || (r->niwant && !r->iwant) ||
        (r->ngraft && !r->graft) || (r->nprune && !r->prune) || (r->nids && !r->ids) || (r->npx && !r->px))
        return false;
    for (uint32_t k = 0; k < r->nihave; ++k)
        if ((uint64_t)r->ihave[k].id0 + r->ihave[k].nid > r->nids) return false;
    for (uint32_t k = 0; k < r->niwant; ++k)
        if ((uint64_t)r->iwant[k].id0 + r->iwant[k].nid > r->nids) return false;
    for (uint32_t k = 0; k < r->nprune; ++k)
        if ((uint64_t)r->prune[k].px0 + r->prune[k].npx > r->npx) return false;
    return true;
}

// fragmentMessageIds (gossipsub.go:1298-1318): buckets of ids whose summed
// (length + 2) stays within limit; an id that alone exceeds it is dropped.
std::vector<std::vector<uint32_t>> fragment_ids(const gsim_wire_rpc& r, const std::vector<uint32_t>& ids, int64_t limit)
{
    constexpr int64_t kOverhead = 2;
    std::vector<std::vector<uint32_t>> out(1);
    int64_t bucket_len = 0;
    for (uint32_t k : ids) {
        const int64_t size = (int64_t)r.ids[k].n + kOverhead;
        if (size > limit) continue;                        // logged and removed by the reference
        bucket_len += size;
        if (bucket_len > limit) {
            out.emplace_back();
            bucket_len = size;
        }
        out.back().push_back(k);
    }
    return out;
}

// ---- decoding (rpc.pb.go's generated Unmarshal, restated) ------------------

// A reader over one message's bytes, with the generated code's checks:
// varints of at most 64 bits, lengths inside the buffer.
struct Rd {
    const uint8_t* p;
    const uint8_t* e;
    bool ok = true;
    bool more() const { return ok && p < e; }
    uint64_t varint()
    {
        uint64_t v = 0;
        for (int s = 0; s < 64; s += 7) {
            if (p >= e) { ok = false; return 0; }            // io.ErrUnexpectedEOF
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << s;
            if (!(b & 0x80)) return v;
        }
        ok = false;                                          // ErrIntOverflow
        return 0;
    }
    // a length-delimited body
    bool body(const uint8_t** q, uint64_t* n)
    {
        const uint64_t L = varint();
        if (!ok || L > (uint64_t)(e - p)) { ok = false; return false; }   // ErrInvalidLength / EOF
        *q = p;
        *n = L;
        p += L;
        return true;
    }
    // skip<Msg>: an unknown field's value (groups nest; an end-group at depth 0 is an error)
    bool skip(int wt)
    {
        int depth = 0;
        for (;;) {
            switch (wt) {
            case 0: varint(); break;
            case 1: if (e - p < 8) ok = false; else p += 8; break;
            case 5: if (e - p < 4) ok = false; else p += 4; break;
            case 2: { const uint8_t* q; uint64_t n; body(&q, &n); break; }
            case 3: ++depth; break;
            case 4: if (depth == 0) ok = false; else --depth; break;   // ErrUnexpectedEndOfGroup
            default: ok = false;                                       // illegal wireType
            }
            if (!ok || depth == 0) return ok;
            const uint64_t k = varint();                     // the group's next field
            if (!ok) return false;
            wt = (int)(k & 7);                               // (skipRpc takes any field number here)
        }
    }
    // the next field's number and wire type (tag checks of the generated code,
    // rpc.pb.go:1345-1352: fieldNum := int32(wire >> 3), so a number above
    // 2^31 is illegal and one of 2^32 + f is field f)
    bool tag(uint32_t* f, int* wt)
    {
        const uint64_t k = varint();
        if (!ok) return false;
        *wt = (int)(k & 7);
        const int32_t fn = (int32_t)(uint32_t)(k >> 3);
        if (*wt == 4 || fn <= 0) { ok = false; return false; }   // end group for non-group / illegal tag
        *f = (uint32_t)fn;
        return true;
    }
};

// Two passes over the same bytes: counting (t == nullptr) then filling.
struct Dec {
    gsim_wire_tables* t;
    uint32_t nsubs = 0, nmsgs = 0, nihave = 0, niwant = 0, ngraft = 0, nprune = 0, nids = 0, npx = 0;
    bool has_control = false;

    static gsim_bytes view(const uint8_t* q, uint64_t n) { return gsim_bytes{q, (uint32_t)n}; }

    // a bytes / string field: present, last occurrence wins
    static bool bytes_field(Rd& r, int wt, gsim_bytes* out)
    {
        if (wt != 2) return false;                           // "wrong wireType"
        const uint8_t* q;
        uint64_t n;
        if (!r.body(&q, &n) || n > 0xFFFFFFFFull) return false;
        if (out) *out = view(q, n);
        return true;
    }

    bool sub(const uint8_t* q, uint64_t n)                   // RPC.SubOpts
    {
        gsim_wire_sub x{-1, {nullptr, 0}};
        Rd r{q, q + n};
        uint32_t f;
        int wt;
        while (r.more()) {
            if (!r.tag(&f, &wt)) return false;
            if (f == 1) {
                if (wt != 0) return false;
                const uint64_t v = r.varint();
                x.subscribe = v != 0 ? 1 : 0;
            } else if (f == 2) {
                if (!bytes_field(r, wt, &x.topic)) return false;
            } else if (!r.skip(wt)) {
                return false;
            }
        }
        if (!r.ok) return false;
        if (t) t->subs[nsubs] = x;
        ++nsubs;
        return true;
    }

    bool msg(const uint8_t* q, uint64_t n)                   // Message
    {
        gsim_wire_msg x{};
        Rd r{q, q + n};
        uint32_t f;
        int wt;
        while (r.more()) {
            if (!r.tag(&f, &wt)) return false;
            gsim_bytes* dst = f == 1 ? &x.from : f == 2 ? &x.data : f == 3 ? &x.seqno : f == 4 ? &x.topic
                            : f == 5 ? &x.signature : f == 6 ? &x.key : nullptr;
            if (dst) {
                if (!bytes_field(r, wt, dst)) return false;
            } else if (!r.skip(wt)) {
                return false;
            }
        }
        if (!r.ok) return false;
        if (t) t->msgs[nmsgs] = x;
        ++nmsgs;
        return true;
    }

    // ControlIHave (id field 2, topic 1) / ControlIWant (id field 1, no topic)
    bool gossip(const uint8_t* q, uint64_t n, bool ihave)
    {
        const uint32_t id_field = ihave ? 2 : 1;
        gsim_bytes topic{nullptr, 0};
        const uint32_t id0 = nids;
        Rd r{q, q + n};
        uint32_t f;
        int wt;
        while (r.more()) {
            if (!r.tag(&f, &wt)) return false;
            if (f == id_field) {
                gsim_bytes b;
                if (!bytes_field(r, wt, &b)) return false;
                if (t) t->ids[nids] = b;
                ++nids;
            } else if (ihave && f == 1) {
                if (!bytes_field(r, wt, &topic)) return false;
            } else if (!r.skip(wt)) {
                return false;
            }
        }
        if (!r.ok) return false;
        if (ihave) {
            if (t) t->ihave[nihave] = gsim_wire_ihave{topic, id0, nids - id0};
            ++nihave;
        } else {
            if (t) t->iwant[niwant] = gsim_wire_iwant{id0, nids - id0};
            ++niwant;
        }
        return true;
    }

    bool graft(const uint8_t* q, uint64_t n)                 // ControlGraft
    {
        gsim_wire_graft x{{nullptr, 0}};
        Rd r{q, q + n};
        uint32_t f;
        int wt;
        while (r.more()) {
            if (!r.tag(&f, &wt)) return false;
            if (f == 1) {
                if (!bytes_field(r, wt, &x.topic)) return false;
            } else if (!r.skip(wt)) {
                return false;
            }
        }
        if (!r.ok) return false;
        if (t) t->graft[ngraft] = x;
        ++ngraft;
        return true;
    }

    bool peer(const uint8_t* q, uint64_t n)                  // PeerInfo
    {
        gsim_wire_px x{};
        Rd r{q, q + n};
        uint32_t f;
        int wt;
        while (r.more()) {
            if (!r.tag(&f, &wt)) return false;
            gsim_bytes* dst = f == 1 ? &x.peer : f == 2 ? &x.record : nullptr;
            if (dst) {
                if (!bytes_field(r, wt, dst)) return false;
            } else if (!r.skip(wt)) {
                return false;
            }
        }
        if (!r.ok) return false;
        if (t) t->px[npx] = x;
        ++npx;
        return true;
    }

    bool prune(const uint8_t* q, uint64_t n)                 // ControlPrune
    {
        gsim_wire_prune x{{nullptr, 0}, npx, 0, 0, 0};
        Rd r{q, q + n};
        uint32_t f;
        int wt;
        while (r.more()) {
            if (!r.tag(&f, &wt)) return false;
            if (f == 1) {
                if (!bytes_field(r, wt, &x.topic)) return false;
            } else if (f == 2) {
                const uint8_t* b;
                uint64_t bn;
                if (wt != 2 || !r.body(&b, &bn) || !peer(b, bn)) return false;
            } else if (f == 3) {
                if (wt != 0) return false;
                x.backoff = r.varint();
                x.has_backoff = 1;
            } else if (!r.skip(wt)) {
                return false;
            }
        }
        if (!r.ok) return false;
        x.npx = npx - x.px0;
        if (t) t->prune[nprune] = x;
        ++nprune;
        return true;
    }

    bool control(const uint8_t* q, uint64_t n)               // ControlMessage (merged)
    {
        has_control = true;
        Rd r{q, q + n};
        uint32_t f;
        int wt;
        while (r.more()) {
            if (!r.tag(&f, &wt)) return false;
            if (f >= 1 && f <= 4) {
                const uint8_t* b;
                uint64_t bn;
                if (wt != 2 || !r.body(&b, &bn)) return false;
                const bool ok = f == 1 ? gossip(b, bn, true) : f == 2 ? gossip(b, bn, false)
                              : f == 3 ? graft(b, bn) : prune(b, bn);
                if (!ok) return false;
            } else if (!r.skip(wt)) {
                return false;
            }
        }
        return r.ok;
    }

    bool rpc(const uint8_t* q, uint64_t n)                   // RPC
    {
        Rd r{q, q + n};
        uint32_t f;
        int wt;
        while (r.more()) {
            if (!r.tag(&f, &wt)) return false;
            if (f >= 1 && f <= 3) {
                const uint8_t* b;
                uint64_t bn;
                if (wt != 2 || !r.body(&b, &bn)) return false;
                const bool ok = f == 1 ? sub(b, bn) : f == 2 ? msg(b, bn) : control(b, bn);
                if (!ok) return false;
            } else if (!r.skip(wt)) {
                return false;
            }
        }
        return r.ok;
    }
};

}  // namespace

extern "C" {

int gsim_wire_decode(const uint8_t* in, uint64_t len, gsim_wire_tables* t, gsim_wire_rpc* rpc)
{
    if (!rpc || !t || (len && !in)) return GSIM_EINVAL;
    *rpc = gsim_wire_rpc{};
    Dec count{nullptr};
    if (!count.rpc(in, len)) return GSIM_EINVAL;
    rpc->nsubs = count.nsubs;
    rpc->nmsgs = count.nmsgs;
    rpc->nihave = count.nihave;
    rpc->niwant = count.niwant;
    rpc->ngraft = count.ngraft;
    rpc->nprune = count.nprune;
    rpc->nids = count.nids;
    rpc->npx = count.npx;
    rpc->has_control = count.has_control ? 1 : 0;
    if (count.nsubs > t->subs_cap || count.nmsgs > t->msgs_cap || count.nihave > t->ihave_cap ||
        count.niwant > t->iwant_cap || count.ngraft > t->graft_cap || count.nprune > t->prune_cap ||
        count.nids > t->ids_cap || count.npx > t->px_cap)
        return GSIM_ERANGE;
    if ((count.nsubs && !t->subs) || (count.nmsgs && !t->msgs) || (count.nihave && !t->ihave) ||
        (count.niwant && !t->iwant) || (count.ngraft && !t->graft) || (count.nprune && !t->prune) ||
        (count.nids && !t->ids) || (count.npx && !t->px))
        return GSIM_EINVAL;
    Dec fill{t};
    fill.rpc(in, len);
    rpc->subs = t->subs;
    rpc->msgs = t->msgs;
    rpc->ihave = t->ihave;
    rpc->iwant = t->iwant;
    rpc->graft = t->graft;
    rpc->prune = t->prune;
    rpc->ids = t->ids;
    rpc->px = t->px;
    return GSIM_OK;
}

int gsim_wire_frames(const uint8_t* in, uint64_t len, uint64_t max_size, uint64_t* off, uint64_t* lens, int32_t cap,
                     int32_t* n, uint64_t* consumed)
{
    if (!n || !consumed || cap < 0 || (cap && (!off || !lens)) || (len && !in)) return GSIM_EINVAL;
    *n = 0;
    *consumed = 0;
    uint64_t pos = 0;
    while (pos < len) {
        // msgio's uvarint length prefix
        uint64_t L = 0, q = pos;
        int s = 0;
        bool done = false;
        while (q < len) {
            const uint8_t b = in[q++];
            if (s >= 64 || (s == 63 && b > 1)) return GSIM_EINVAL;   // binary.ErrOverflow
            L |= (uint64_t)(b & 0x7F) << s;
            s += 7;
            if (!(b & 0x80)) { done = true; break; }
        }
        if (!done) break;                                    // the prefix is still arriving
        if (L > max_size) return GSIM_ERANGE;                // msgio.ErrMsgTooLarge
        if (len - q < L) break;                              // the body is still arriving
        if (*n >= cap) return GSIM_ERANGE;
        off[*n] = q;
        lens[*n] = L;
        ++*n;
        pos = q + L;
        *consumed = pos;
    }
    return GSIM_OK;
}

uint64_t gsim_wire_size(const gsim_wire_rpc* rpc)
{
    if (!tables_ok(rpc)) return 0;
    return frag_size(*rpc, whole(*rpc));
}

int gsim_wire_encode(const gsim_wire_rpc* rpc, uint8_t* out, uint64_t cap, uint64_t* len)
{
    if (!tables_ok(rpc) || !len || (cap && !out)) return GSIM_EINVAL;
    const Frag f = whole(*rpc);
    const uint64_t n = frag_size(*rpc, f);
    *len = n;
    if (n > cap) return GSIM_ERANGE;
    Writer w{out};
    write_frag(w, *rpc, f);
    return GSIM_OK;
}

int gsim_wire_fragment(const gsim_wire_rpc* rpc, int64_t limit, uint8_t* out, uint64_t cap, uint64_t* len,
                       uint64_t* off, int32_t max_frags, int32_t* nfrags)
{
    if (!tables_ok(rpc) || !len || !nfrags || limit <= 0 || max_frags < 0 || (max_frags && !off) || (cap && !out))
        return GSIM_EINVAL;
    const gsim_wire_rpc& r = *rpc;
    const Frag in = whole(r);
    std::vector<Frag> rpcs;
    if ((int64_t)frag_size(r, in) < limit) {
        rpcs.push_back(in);
    } else {
        rpcs.emplace_back();
        // outRPC: the last fragment if it fits sizeToAdd (+1 for the field
        // tag) more bytes, else a new one; withCtl: with a control message
        auto out_rpc = [&](uint64_t size_to_add, bool with_ctl) -> Frag& {
            Frag& cur = rpcs.back();
            if ((int64_t)(frag_size(r, cur) + size_to_add + 1) < limit) {
                if (with_ctl) cur.has_control = true;
                return cur;
            }
            rpcs.emplace_back();
            rpcs.back().has_control = with_ctl;
            return rpcs.back();
        };
        for (uint32_t k : in.msgs) {
            const uint64_t s = msg_size(r.msgs[k]);
            if ((int64_t)s > limit) return GSIM_EINVAL;    // "message with len=%d exceeds limit %d"
            out_rpc(s, false).msgs.push_back(k);
        }
        for (uint32_t k : in.subs) out_rpc(sub_size(r.subs[k]), false).subs.push_back(k);
        if (in.has_control) {
            // all control in one more RPC when it fits
            Frag ctl;
            ctl.has_control = true;
            ctl.ihave = in.ihave;
            ctl.iwant = in.iwant;
            ctl.graft = in.graft;
            ctl.prune = in.prune;
            if ((int64_t)frag_size(r, ctl) < limit) {
                rpcs.push_back(std::move(ctl));
            } else {
                for (uint32_t k : in.graft) out_rpc(graft_size(r.graft[k]), true).graft.push_back(k);
                for (uint32_t k : in.prune) out_rpc(prune_size(r, r.prune[k]), true).prune.push_back(k);
                constexpr int64_t kOverhead = 6;
                for (const auto& g : in.iwant)
                    for (auto& ids : fragment_ids(r, g.ids, limit - kOverhead)) {
                        Gossip x{false, {nullptr, 0}, std::move(ids)};
                        out_rpc(gossip_size(r, x), true).iwant.push_back(std::move(x));
                    }
                for (const auto& g : in.ihave)
                    for (auto& ids : fragment_ids(r, g.ids, limit - kOverhead)) {
                        Gossip x{false, {nullptr, 0}, std::move(ids)};   // the topic id is not carried over
                        out_rpc(gossip_size(r, x), true).ihave.push_back(std::move(x));
                    }
            }
        }
    }
    uint64_t total = 0;
    for (const auto& f : rpcs) total += frag_size(r, f);
    *len = total;
    *nfrags = (int32_t)rpcs.size();
    if (total > cap || (int64_t)rpcs.size() > max_frags) return GSIM_ERANGE;
    Writer w{out};
    uint64_t pos = 0;
    for (size_t k = 0; k < rpcs.size(); ++k) {
        off[k] = pos;
        write_frag(w, r, rpcs[k]);
        pos = (uint64_t)(w.p - out);
    }
    off[rpcs.size()] = pos;
    return GSIM_OK;
}

}  // extern "C"
