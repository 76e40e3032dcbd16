"""CPU restatement of the GossipSub wire format — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this; the product path (libgsim's gsim_wire_*) never
does.  Two independent pieces check the library's encoders:

* `pb()`: protobuf message classes built at run time from a descriptor that
  restates the schema of pb/rpc.proto:5-57 (proto2; field names, numbers and
  labels as there).  The serializer is the protobuf runtime's own — an
  encoder written by others, not ours.  The id fields declared `string` in
  rpc.proto are declared `bytes` here: same wire type (length-delimited), no
  UTF-8 check (the reference's own comment: Go emits invalid UTF-8 there).
* `fragment_rpc` / `fragment_message_ids`: fragmentRPC restated from
  gossipsub.go:1204-1296 and fragmentMessageIds from 1298-1318, on those
  classes (Size() = ByteSize()).

Parity: the restatement is pinned by the reference's own test,
TestFragmentRPCFunction (gossipsub_test.go:2338-2500), restated in
tests/test_wire.py against both this module and the library.
"""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_CLASSES = None


def pb():
    """{name: class} for RPC, RPC.SubOpts, Message, ControlMessage,
    ControlIHave, ControlIWant, ControlGraft, ControlPrune, PeerInfo."""
    global _CLASSES
    if _CLASSES is not None:
        return _CLASSES
    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="gsim_test_rpc.proto", package="gsimtest.pb", syntax="proto2")

    def msg(name, fields, parent=None):
        m = (parent.nested_type if parent is not None else fdp.message_type).add(name=name)
        for (fname, num, label, typ, tname) in fields:
            f = m.field.add(name=fname, number=num, label=label, type=typ)
            if tname:
                f.type_name = tname
        return m

    OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    B, S, BOOL, U64, M = F.TYPE_BYTES, F.TYPE_STRING, F.TYPE_BOOL, F.TYPE_UINT64, F.TYPE_MESSAGE
    rpc = msg("RPC", [("subscriptions", 1, REP, M, ".gsimtest.pb.RPC.SubOpts"),
                      ("publish", 2, REP, M, ".gsimtest.pb.Message"),
                      ("control", 3, OPT, M, ".gsimtest.pb.ControlMessage")])
    msg("SubOpts", [("subscribe", 1, OPT, BOOL, None), ("topicid", 2, OPT, B, None)], parent=rpc)
    msg("Message", [("from", 1, OPT, B, None), ("data", 2, OPT, B, None), ("seqno", 3, OPT, B, None),
                    ("topic", 4, OPT, B, None), ("signature", 5, OPT, B, None), ("key", 6, OPT, B, None)])
    msg("ControlMessage", [("ihave", 1, REP, M, ".gsimtest.pb.ControlIHave"),
                           ("iwant", 2, REP, M, ".gsimtest.pb.ControlIWant"),
                           ("graft", 3, REP, M, ".gsimtest.pb.ControlGraft"),
                           ("prune", 4, REP, M, ".gsimtest.pb.ControlPrune")])
    msg("ControlIHave", [("topicID", 1, OPT, B, None), ("messageIDs", 2, REP, B, None)])
    msg("ControlIWant", [("messageIDs", 1, REP, B, None)])
    msg("ControlGraft", [("topicID", 1, OPT, B, None)])
    msg("ControlPrune", [("topicID", 1, OPT, B, None), ("peers", 2, REP, M, ".gsimtest.pb.PeerInfo"),
                         ("backoff", 3, OPT, U64, None)])
    msg("PeerInfo", [("peerID", 1, OPT, B, None), ("signedPeerRecord", 2, OPT, B, None)])
    del S
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    names = ["RPC", "RPC.SubOpts", "Message", "ControlMessage", "ControlIHave", "ControlIWant", "ControlGraft",
             "ControlPrune", "PeerInfo"]
    _CLASSES = {n: message_factory.GetMessageClass(pool.FindMessageTypeByName("gsimtest.pb." + n)) for n in names}
    return _CLASSES


_TRACE = None


def trace_pb():
    """{name: class} for TraceEvent and TraceEventBatch, from a descriptor
    restating pb/trace.proto:5-150 for the events the engine produces
    (PublishMessage, RejectMessage, DuplicateMessage, DeliverMessage,
    AddPeer, RemovePeer, RecvRPC, SendRPC, DropRPC with their RPCMeta, Join,
    Leave, Graft, Prune; field names, numbers, types as there).  Serialized by
    the protobuf runtime."""
    global _TRACE
    if _TRACE is not None:
        return _TRACE
    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="gsim_test_trace.proto", package="gsimtest.tr", syntax="proto2")
    OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    B, S, I64, E, M = F.TYPE_BYTES, F.TYPE_STRING, F.TYPE_INT64, F.TYPE_ENUM, F.TYPE_MESSAGE
    ev = fdp.message_type.add(name="TraceEvent")
    ty = ev.enum_type.add(name="Type")
    for k, name in enumerate(["PUBLISH_MESSAGE", "REJECT_MESSAGE", "DUPLICATE_MESSAGE", "DELIVER_MESSAGE", "ADD_PEER",
                              "REMOVE_PEER", "RECV_RPC", "SEND_RPC", "DROP_RPC", "JOIN", "LEAVE", "GRAFT", "PRUNE"]):
        ty.value.add(name=name, number=k)
    T = ".gsimtest.tr.TraceEvent."
    for (fname, num, label, typ, tname) in [("type", 1, OPT, E, T + "Type"), ("peerID", 2, OPT, B, None),
                                            ("timestamp", 3, OPT, I64, None),
                                            ("publishMessage", 4, OPT, M, T + "PublishMessage"),
                                            ("rejectMessage", 5, OPT, M, T + "RejectMessage"),
                                            ("duplicateMessage", 6, OPT, M, T + "DuplicateMessage"),
                                            ("deliverMessage", 7, OPT, M, T + "DeliverMessage"),
                                            ("addPeer", 8, OPT, M, T + "AddPeer"),
                                            ("removePeer", 9, OPT, M, T + "RemovePeer"),
                                            ("recvRPC", 10, OPT, M, T + "RecvRPC"),
                                            ("sendRPC", 11, OPT, M, T + "SendRPC"),
                                            ("dropRPC", 12, OPT, M, T + "DropRPC"),
                                            ("join", 13, OPT, M, T + "Join"), ("leave", 14, OPT, M, T + "Leave"),
                                            ("graft", 15, OPT, M, T + "Graft"), ("prune", 16, OPT, M, T + "Prune")]:
        f = ev.field.add(name=fname, number=num, label=label, type=typ)
        if tname:
            f.type_name = tname

    def sub(name, fields):
        m = ev.nested_type.add(name=name)
        for fd in fields:
            fname, num, typ = fd[:3]
            f = m.field.add(name=fname, number=num, label=fd[3] if len(fd) > 3 else OPT, type=typ)
            if len(fd) > 4:
                f.type_name = T + fd[4]

    BOOL = F.TYPE_BOOL
    # RPCMeta and its parts (pb/trace.proto:107-146); RecvRPC / SendRPC / DropRPC (76-89)
    sub("MessageMeta", [("messageID", 1, B), ("topic", 2, S)])
    sub("SubMeta", [("subscribe", 1, BOOL), ("topic", 2, S)])
    sub("ControlIHaveMeta", [("topic", 1, S), ("messageIDs", 2, B, REP)])
    sub("ControlIWantMeta", [("messageIDs", 1, B, REP)])
    sub("ControlGraftMeta", [("topic", 1, S)])
    sub("ControlPruneMeta", [("topic", 1, S), ("peers", 2, B, REP)])
    sub("ControlMeta", [("ihave", 1, M, REP, "ControlIHaveMeta"), ("iwant", 2, M, REP, "ControlIWantMeta"),
                        ("graft", 3, M, REP, "ControlGraftMeta"), ("prune", 4, M, REP, "ControlPruneMeta")])
    sub("RPCMeta", [("messages", 1, M, REP, "MessageMeta"), ("subscription", 2, M, REP, "SubMeta"),
                    ("control", 3, M, OPT, "ControlMeta")])
    sub("RecvRPC", [("receivedFrom", 1, B), ("meta", 2, M, OPT, "RPCMeta")])
    sub("SendRPC", [("sendTo", 1, B), ("meta", 2, M, OPT, "RPCMeta")])
    sub("DropRPC", [("sendTo", 1, B), ("meta", 2, M, OPT, "RPCMeta")])

    sub("PublishMessage", [("messageID", 1, B), ("topic", 2, S)])
    sub("RejectMessage", [("messageID", 1, B), ("receivedFrom", 2, B), ("reason", 3, S), ("topic", 4, S)])
    sub("DuplicateMessage", [("messageID", 1, B), ("receivedFrom", 2, B), ("topic", 3, S)])
    sub("DeliverMessage", [("messageID", 1, B), ("topic", 2, S), ("receivedFrom", 3, B)])
    sub("AddPeer", [("peerID", 1, B), ("proto", 2, S)])
    sub("RemovePeer", [("peerID", 1, B)])
    sub("Join", [("topic", 1, S)])
    sub("Leave", [("topic", 2, S)])             # pb/trace.proto:92-94: Leave.topic is field 2
    sub("Graft", [("peerID", 1, B), ("topic", 2, S)])
    sub("Prune", [("peerID", 1, B), ("topic", 2, S)])
    b = fdp.message_type.add(name="TraceEventBatch")
    b.field.add(name="batch", number=1, label=REP, type=M, type_name=".gsimtest.tr.TraceEvent")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    _TRACE = {n: message_factory.GetMessageClass(pool.FindMessageTypeByName("gsimtest.tr." + n))
              for n in ["TraceEvent", "TraceEventBatch"]}
    return _TRACE


class FragmentError(ValueError):
    pass


def fragment_message_ids(msg_ids, limit):
    """fragmentMessageIds (gossipsub.go:1298-1318)."""
    overhead = 2                                    # protobuf overhead per array element
    out = [[]]
    bucket_len = 0
    for mid in msg_ids:
        size = len(mid) + overhead
        if size > limit:                            # pathological: removed from the outgoing gossip
            continue
        bucket_len += size
        if bucket_len > limit:
            out.append([])
            bucket_len = size
        out[-1].append(mid)
    return out


def fragment_rpc(rpc, limit):
    """fragmentRPC (gossipsub.go:1204-1296) on pb() RPC objects."""
    C = pb()
    if rpc.ByteSize() < limit:
        return [rpc]
    rpcs = [C["RPC"]()]

    def out_rpc(size_to_add, with_ctl):            # outRPC (1218-1236)
        cur = rpcs[-1]
        if cur.ByteSize() + size_to_add + 1 < limit:
            if with_ctl and not cur.HasField("control"):
                cur.control.SetInParent()
            return cur
        nxt = C["RPC"]()
        if with_ctl:
            nxt.control.SetInParent()
        rpcs.append(nxt)
        return nxt

    for m in rpc.publish:                          # 1238-1246
        s = m.ByteSize()
        if s > limit:
            raise FragmentError(f"message with len={s} exceeds limit {limit}")
        out_rpc(s, False).publish.add().CopyFrom(m)
    for sub in rpc.subscriptions:                  # 1248-1251
        out_rpc(sub.ByteSize(), False).subscriptions.add().CopyFrom(sub)
    if not rpc.HasField("control"):                # 1253-1257
        return rpcs
    ctl = rpc.control
    ctl_out = C["RPC"]()                           # 1259-1264
    ctl_out.control.CopyFrom(ctl)
    if ctl_out.ByteSize() < limit:
        rpcs.append(ctl_out)
        return rpcs
    for g in ctl.graft:                            # 1266-1274
        out_rpc(g.ByteSize(), True).control.graft.add().CopyFrom(g)
    for p in ctl.prune:
        out_rpc(p.ByteSize(), True).control.prune.add().CopyFrom(p)
    overhead = 6                                   # 1279-1295
    for iw in ctl.iwant:
        for ids in fragment_message_ids(list(iw.messageIDs), limit - overhead):
            x = C["ControlIWant"](messageIDs=ids)
            out_rpc(x.ByteSize(), True).control.iwant.add().CopyFrom(x)
    for ih in ctl.ihave:
        for ids in fragment_message_ids(list(ih.messageIDs), limit - overhead):
            x = C["ControlIHave"](messageIDs=ids)  # the topic id is not carried over
            out_rpc(x.ByteSize(), True).control.ihave.add().CopyFrom(x)
    return rpcs


def trace_rpc_meta(rpc, meta):
    """traceRPCMeta (trace.go:326-414) restated: fill the TraceEvent.RPCMeta
    `meta` from a decoded RPC (pb() classes).  Message ids are
    DefaultMsgIdFn's from || seqno (pubsub.go); optional fields are copied when
    present (Go copies the pointers); the control meta exists whenever the RPC
    has a control message; a PRUNE's peers are its PeerInfo ids (an absent id
    is an empty one)."""
    for m in rpc.publish:
        mm = meta.messages.add()
        mm.messageID = getattr(m, "from") + m.seqno
        if m.HasField("topic"):
            mm.topic = m.topic.decode("utf-8", "surrogateescape")
    for sub in rpc.subscriptions:
        sm = meta.subscription.add()
        if sub.HasField("subscribe"):
            sm.subscribe = sub.subscribe
        if sub.HasField("topicid"):
            sm.topic = sub.topicid.decode("utf-8", "surrogateescape")
    if rpc.HasField("control"):
        c = meta.control
        c.SetInParent()
        for ih in rpc.control.ihave:
            x = c.ihave.add()
            if ih.HasField("topicID"):
                x.topic = ih.topicID.decode("utf-8", "surrogateescape")
            x.messageIDs.extend(ih.messageIDs)
        for iw in rpc.control.iwant:
            c.iwant.add().messageIDs.extend(iw.messageIDs)
        for g in rpc.control.graft:
            x = c.graft.add()
            if g.HasField("topicID"):
                x.topic = g.topicID.decode("utf-8", "surrogateescape")
        for p in rpc.control.prune:
            x = c.prune.add()
            if p.HasField("topicID"):
                x.topic = p.topicID.decode("utf-8", "surrogateescape")
            x.peers.extend([pi.peerID for pi in p.peers])


def trace_rpc_events(rpcs, peer_id, timestamp, which):
    """The TraceEventBatch pubsubTracer's SendRPC / RecvRPC / DropRPC
    (trace.go:250-324) would write for encoded RPCs [(from, to, bytes)]: per
    RPC, SEND_RPC at the sender (bit 0 of which), RECV_RPC at the receiver
    (bit 1), DROP_RPC at the sender (bit 2)."""
    P, T = pb(), trace_pb()
    batch = T["TraceEventBatch"]()
    for (frm, to, raw) in rpcs:
        rpc = P["RPC"]()
        rpc.ParseFromString(raw)
        for bit, (typ, field, me, other) in enumerate([(7, "sendRPC", frm, to), (6, "recvRPC", to, frm),
                                                       (8, "dropRPC", frm, to)]):
            if not (which >> bit) & 1:
                continue
            ev = batch.batch.add()
            ev.type = typ
            ev.peerID = peer_id(me)
            ev.timestamp = timestamp
            body = getattr(ev, field)
            if field == "recvRPC":
                body.receivedFrom = peer_id(other)
            else:
                body.sendTo = peer_id(other)
            trace_rpc_meta(rpc, body.meta)
            body.meta.SetInParent()
    return batch.SerializeToString()
