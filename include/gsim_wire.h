/* gsim_wire.h — the GossipSub wire format.
 *
 * Two halves:
 *
 *   1. Host encoders of the reference's protobuf messages (pb/rpc.proto:5-57,
 *      proto2, gogo-protobuf field order) and its fragmentRPC
 *      (gossipsub.go:1204-1318).  An RPC is described by flat tables; every
 *      optional field is present when its pointer is non-NULL (an empty byte
 *      string with a non-NULL pointer is encoded, as Go encodes a non-nil
 *      empty slice).
 *
 *   2. gsim_wire_heartbeat: the RPCs the engine's routers send at a
 *      heartbeat — GRAFT/PRUNE (sendGraftPrune, gossipsub.go:1672-1709) with
 *      the IHAVE gossip piggybacked on them (emitGossip + piggybackGossip,
 *      gossipsub.go:1711-1816), or the IHAVE gossip alone (flush,
 *      gossipsub.go:1777-1791) — encoded on the device for a range of
 *      senders, one RPC per (sender, receiver) edge that carries any.
 *
 * Orders the reference leaves to Go map iteration are fixed here: topics
 * ascend by index in every control list; a topic's IHAVE ids follow
 * mcache.GetGossipIDs (mcache.go:82-92: newest history window first, each
 * window in Put order — within a round the origin's own publication first,
 * then receipts by (first sender, message id)).
 */
#ifndef GSIM_WIRE_H
#define GSIM_WIRE_H

#include <stddef.h>
#include <stdint.h>

#include "gsim.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A byte string; absent (optional field not set) when p is NULL. */
typedef struct gsim_bytes {
    const uint8_t* p;
    uint32_t n;
} gsim_bytes;

/* RPC.SubOpts (rpc.proto:8-11): subscribe < 0 = absent. */
typedef struct gsim_wire_sub {
    int32_t subscribe;
    gsim_bytes topic;
} gsim_wire_sub;

/* Message (rpc.proto:16-23). */
typedef struct gsim_wire_msg {
    gsim_bytes from, data, seqno, topic, signature, key;
} gsim_wire_msg;

/* ControlIHave (rpc.proto:32-36): message ids ids[id0 .. id0 + nid). */
typedef struct gsim_wire_ihave {
    gsim_bytes topic;
    uint32_t id0, nid;
} gsim_wire_ihave;

/* ControlIWant (rpc.proto:38-41). */
typedef struct gsim_wire_iwant {
    uint32_t id0, nid;
} gsim_wire_iwant;

/* ControlGraft (rpc.proto:43-45). */
typedef struct gsim_wire_graft {
    gsim_bytes topic;
} gsim_wire_graft;

/* PeerInfo (rpc.proto:53-56). */
typedef struct gsim_wire_px {
    gsim_bytes peer, record;
} gsim_wire_px;

/* ControlPrune (rpc.proto:47-51): peers px[px0 .. px0 + npx); has_backoff 0 =
 * Backoff absent. */
typedef struct gsim_wire_prune {
    gsim_bytes topic;
    uint32_t px0, npx;
    int32_t has_backoff;
    uint64_t backoff;
} gsim_wire_prune;

/* RPC (rpc.proto:5-14).  has_control: the ControlMessage is present (Go:
 * Control != nil), even when all its lists are empty. */
typedef struct gsim_wire_rpc {
    const gsim_wire_sub* subs;
    uint32_t nsubs;
    const gsim_wire_msg* msgs;
    uint32_t nmsgs;
    int32_t has_control;
    const gsim_wire_ihave* ihave;
    uint32_t nihave;
    const gsim_wire_iwant* iwant;
    uint32_t niwant;
    const gsim_wire_graft* graft;
    uint32_t ngraft;
    const gsim_wire_prune* prune;
    uint32_t nprune;
    const gsim_bytes* ids;       /* message-id table of ihave / iwant */
    uint32_t nids;
    const gsim_wire_px* px;      /* PeerInfo table of prune */
    uint32_t npx;
} gsim_wire_rpc;

/* RPC.Size() (rpc.pb.go): encoded length in bytes. */
uint64_t gsim_wire_size(const gsim_wire_rpc* rpc);

/* RPC.Marshal(): writes gsim_wire_size(rpc) bytes to out.  GSIM_ERANGE when
 * cap is too small (*len = the size needed). */
int gsim_wire_encode(const gsim_wire_rpc* rpc, uint8_t* out, uint64_t cap, uint64_t* len);

/* fragmentRPC(rpc, limit) (gossipsub.go:1204-1296, with fragmentMessageIds
 * 1298-1318), its quirks kept: a fragmented IHAVE loses its topic id; a
 * message id longer than the limit is dropped; an RPC that fits (Size() <
 * limit) is returned whole.  The fragments are encoded back to back in out;
 * off[k] .. off[k+1] is fragment k (off has room for max_frags + 1 entries).
 * GSIM_EINVAL when a published message alone exceeds the limit (the
 * reference's error), GSIM_ERANGE when out or off is too small (*nfrags and
 * *len then hold what is needed). */
int gsim_wire_fragment(const gsim_wire_rpc* rpc, int64_t limit, uint8_t* out, uint64_t cap, uint64_t* len,
                       uint64_t* off, int32_t max_frags, int32_t* nfrags);

/* ---- decoding: RPC.Unmarshal and the delimited stream --------------------- */

/* Caller-owned tables gsim_wire_decode fills (no allocation crosses the
 * boundary).  Each pointer has room for its *_cap entries. */
typedef struct gsim_wire_tables {
    gsim_wire_sub* subs;
    gsim_wire_msg* msgs;
    gsim_wire_ihave* ihave;
    gsim_wire_iwant* iwant;
    gsim_wire_graft* graft;
    gsim_wire_prune* prune;
    gsim_bytes* ids;
    gsim_wire_px* px;
    uint32_t subs_cap, msgs_cap, ihave_cap, iwant_cap, graft_cap, prune_cap, ids_cap, px_cap;
} gsim_wire_tables;

/* RPC.Unmarshal (rpc.pb.go, gogo-protobuf; called by handleNewStream,
 * comm.go:66-82): decodes one RPC of len bytes into *rpc, whose tables point
 * into t and whose byte strings point into `in` (zero copy: keep `in` alive).
 * Semantics of the generated code: a repeated field appends per occurrence;
 * an optional scalar or bytes field takes its last occurrence; the optional
 * ControlMessage merges every occurrence (its lists concatenate in order);
 * unknown fields (any wire type, groups included) are skipped, not kept
 * (gogo keeps them in XXX_unrecognized, which nothing on the path reads).
 * GSIM_EINVAL for a malformed RPC (truncated field, varint overflow, a known
 * field with the wrong wire type, field number 0, a stray end-group:
 * "bogus rpc" in the reference) with *rpc zeroed; GSIM_ERANGE when a table
 * is too small, with rpc's counts set to the entries needed and its table
 * pointers NULL. */
int gsim_wire_decode(const uint8_t* in, uint64_t len, gsim_wire_tables* t, gsim_wire_rpc* rpc);

/* The varint-delimited stream of RPCs (msgio.NewVarintReaderSize(s,
 * maxMessageSize), comm.go:64-82; the sender's msgio varint writer): splits
 * in[0 .. len) into frames, frame k being the body in[off[k] .. off[k] +
 * lens[k]).  Stops at a trailing incomplete frame (*consumed = the bytes of
 * the whole frames; the rest waits for more input).  GSIM_ERANGE when a
 * frame's length exceeds max_size (msgio.ErrMsgTooLarge: the reference resets
 * the stream) or when more than cap frames are complete (*n = the frames
 * found so far, all returned); GSIM_EINVAL for a length varint over 64 bits. */
int gsim_wire_frames(const uint8_t* in, uint64_t len, uint64_t max_size, uint64_t* off, uint64_t* lens, int32_t cap,
                     int32_t* n, uint64_t* consumed);

/* ---- device: the heartbeat's RPCs ---------------------------------------- */

/* One encoded RPC in the device output. */
typedef struct gsim_wire_ref {
    uint32_t from, to;      /* sender, receiver (network peer ids) */
    uint32_t len;           /* bytes */
    uint32_t pad;
    uint64_t offset;        /* into the output buffer */
} gsim_wire_ref;

/* Names and ids the RPCs carry.
 *   topic_names[t]: ControlIHave/Graft/Prune.topicID of topic t (T entries);
 *   peer_ids / peer_id_len: optional fixed-length peer ids (N x peer_id_len
 *     bytes); a message's id is then peer_id(origin) || seqno (the reference's
 *     DefaultMsgIdFn, pubsub.go: from + seqno), else seqno alone;
 *     the seqno is the gsim_msg id as 8 big-endian bytes;
 *   prune_backoff_s: ControlPrune.Backoff (PruneBackoff / 1s, gossipsub.go:1872).
 * Not encoded, refused instead: a PRUNE that carries peer exchange (doPX,
 * makePrune gossipsub.go:1878-1903: its PX list is not kept per PRUNE) ->
 * GSIM_ESTATE; a gossip window of more than MaxIHaveLength ids (emitGossip's
 * per-target random subsets, 1763-1772) -> GSIM_ESTATE. */
typedef struct gsim_wire_names {
    const gsim_bytes* topic_names;
    const uint8_t* peer_ids;
    uint32_t peer_id_len;
    uint64_t prune_backoff_s;
} gsim_wire_names;

/* Encode, on the device, the RPCs that senders [p0, p1) sent at heartbeat
 * `tick` (call it after gsim_heartbeat(tick) and before the tick's first
 * round).  d_out / d_refs are device buffers of out_cap bytes / ref_cap
 * entries; refs come in sender order, each sender's in its row order.
 * *n_rpcs / *bytes: what was written (GSIM_ERANGE with the totals needed
 * when a buffer is too small; nothing is written then). */
int gsim_wire_heartbeat(gsim_handle* h, int64_t tick, uint32_t p0, uint32_t p1, const gsim_wire_names* names,
                        uint8_t* d_out, uint64_t out_cap, gsim_wire_ref* d_refs, int64_t ref_cap,
                        int64_t* n_rpcs, uint64_t* bytes);

/* TraceEventBatch (pb/trace.proto:148-150) of n trace records from
 * gsim_trace_read (include/gsim.h): one TraceEvent {type, peerID, timestamp,
 * and the event's message} per record, fields in number order as gogo's
 * Marshal writes them (trace.pb.go).  Peer ids come from names->peer_ids (4
 * big-endian bytes of the peer index when peer_id_len is 0), topics from
 * names->topic_names; a messageID is the gsim id as 8 big-endian bytes —
 * the seqno alone, even when peer_ids is given (trace records carry no
 * origin), so with peer ids these messageIDs are NOT the ids
 * gsim_wire_heartbeat's IHAVEs carry (peer_id(origin) || seqno): join the
 * two on the trailing 8 bytes;
 * AddPeer.proto is `proto` (e.g. "/meshsub/1.1.0"); RejectMessage.reason is
 * the reference's string for the verdict (tracer.go:31-38).  *len: the
 * bytes written (GSIM_ERANGE with *len = the size needed when cap is short). */
int gsim_trace_encode(const gsim_trace_event* ev, int64_t n, const gsim_wire_names* names, const char* proto,
                      uint8_t* out, uint64_t cap, uint64_t* len);

/* The RPC-level trace events (pubsubTracer.SendRPC / RecvRPC / DropRPC,
 * trace.go:250-324) of n encoded RPCs — e.g. gsim_wire_heartbeat's output
 * copied to host, with its refs (from, to, offset, len into rpcs).  Per RPC,
 * in ref order, one TraceEvent per bit of `which`: bit 0 SEND_RPC at the
 * sender (sendTo = receiver), bit 1 RECV_RPC at the receiver (receivedFrom =
 * sender), bit 2 DROP_RPC at the sender (the caller decides which RPCs a full
 * queue dropped: the engine models no outbound queue), each with the RPC's
 * RPCMeta as traceRPCMeta builds it (trace.go:326-414: message ids from ||
 * seqno, topics, subscriptions, IHAVE / IWANT ids, GRAFT / PRUNE topics and
 * PX peer ids) and timestamp_ns.  Peer ids as gsim_trace_encode.  Written as
 * a TraceEventBatch; *len the bytes (GSIM_ERANGE with *len = the size needed
 * when cap is short; GSIM_EINVAL for a malformed RPC). */
int gsim_trace_rpc_encode(const uint8_t* rpcs, const gsim_wire_ref* refs, int64_t n, const gsim_wire_names* names,
                          int64_t timestamp_ns, int32_t which, uint8_t* out, uint64_t cap, uint64_t* len);

/* PBTracer's output (tracer.go:130-179): the events of a TraceEventBatch
 * (gsim_trace_encode / gsim_trace_rpc_encode output, len bytes) as the
 * varint-delimited TraceEvent stream protoio's DelimitedWriter writes to the
 * trace file.  *n: the bytes (GSIM_ERANGE with *n = the size needed when cap
 * is short; GSIM_EINVAL for bytes that are not a TraceEventBatch). */
int gsim_trace_delimited(const uint8_t* batch, uint64_t len, uint8_t* out, uint64_t cap, uint64_t* n);

#ifdef __cplusplus
}
#endif

#endif /* GSIM_WIRE_H */
