"""The wire format (include/gsim_wire.h).

CPU part:
  * gsim_wire_encode is byte-identical to the protobuf runtime's serializer
    on the schema of pb/rpc.proto:5-57 (oracle/wire_oracle.py), over random
    RPCs with every field present, absent and empty;
  * gsim_wire_fragment follows fragmentRPC (gossipsub.go:1204-1318): the
    reference's own TestFragmentRPCFunction (gossipsub_test.go:2338-2500) is
    restated against both the library and the Python restatement, and the two
    agree fragment for fragment on random RPCs and limits.
GPU part: gsim_wire_heartbeat, the RPCs the routers send at a heartbeat
encoded on the device, equals the RPCs built on the CPU from the oracle's
heartbeat (GRAFT/PRUNE inbox, emitGossip targets) and from mcache windows
driven by the oracle's Put stream (the pinned orc_mcache, mcache.go).
"""
import os
import sys

import numpy as np
import pytest

from conftest import REPO
from gsim import _abi, wire

sys.path.insert(0, os.path.join(REPO, "oracle"))
import wire_oracle as wo  # noqa: E402  (test infrastructure)


def to_pb(r: wire.RPC):
    C = wo.pb()
    out = C["RPC"]()
    for s in r.subscriptions:
        x = out.subscriptions.add()
        if s.subscribe is not None:
            x.subscribe = bool(s.subscribe)
        if s.topicid is not None:
            x.topicid = wire._b(s.topicid)
    for m in r.publish:
        x = out.publish.add()
        for name, v in (("from", m.from_), ("data", m.data), ("seqno", m.seqno), ("topic", m.topic),
                        ("signature", m.signature), ("key", m.key)):
            if v is not None:
                setattr(x, name, wire._b(v))
    if r.control is not None:
        c = out.control
        c.SetInParent()
        for g in r.control.ihave:
            x = c.ihave.add()
            if g.topicID is not None:
                x.topicID = wire._b(g.topicID)
            x.messageIDs.extend([wire._b(i) for i in g.messageIDs])
        for g in r.control.iwant:
            c.iwant.add().messageIDs.extend([wire._b(i) for i in g.messageIDs])
        for g in r.control.graft:
            x = c.graft.add()
            if g.topicID is not None:
                x.topicID = wire._b(g.topicID)
        for p in r.control.prune:
            x = c.prune.add()
            if p.topicID is not None:
                x.topicID = wire._b(p.topicID)
            for pi in p.peers:
                y = x.peers.add()
                if pi.peerID is not None:
                    y.peerID = pi.peerID
                if pi.signedPeerRecord is not None:
                    y.signedPeerRecord = pi.signedPeerRecord
            if p.backoff is not None:
                x.backoff = p.backoff
    return out


def rand_bytes(rng, lo=0, hi=40, absent=0.2):
    if rng.random() < absent:
        return None
    return rng.bytes(int(rng.integers(lo, hi + 1)))


def rand_rpc(rng, scale=1.0):
    n = lambda k: int(rng.integers(0, max(1, int(k * scale)) + 1))  # noqa: E731
    r = wire.RPC()
    for _ in range(n(3)):
        r.subscriptions.append(wire.SubOpts(None if rng.random() < 0.2 else bool(rng.integers(2)),
                                            rand_bytes(rng, 0, 12)))
    for _ in range(n(4)):
        r.publish.append(wire.Message(*(rand_bytes(rng, 0, int(300 * scale)) for _ in range(6))))
    if rng.random() < 0.8:
        c = wire.ControlMessage()
        for _ in range(n(3)):
            c.ihave.append(wire.ControlIHave(rand_bytes(rng, 0, 10), [rng.bytes(int(rng.integers(0, 50)))
                                                                       for _ in range(n(20))]))
        for _ in range(n(3)):
            c.iwant.append(wire.ControlIWant([rng.bytes(int(rng.integers(0, 50))) for _ in range(n(20))]))
        for _ in range(n(3)):
            c.graft.append(wire.ControlGraft(rand_bytes(rng, 0, 10)))
        for _ in range(n(3)):
            c.prune.append(wire.ControlPrune(rand_bytes(rng, 0, 10),
                                             [wire.PeerInfo(rand_bytes(rng), rand_bytes(rng)) for _ in range(n(2))],
                                             None if rng.random() < 0.3 else int(rng.integers(0, 2**40))))
        r.control = c
    return r


def test_encode_matches_protobuf_runtime():
    rng = np.random.default_rng(1)
    for k in range(400):
        r = rand_rpc(rng, scale=1.0 + (k % 7))
        want = to_pb(r).SerializeToString()
        assert wire.marshal(r) == want, k
        assert wire.size(r) == len(want)


def test_encode_edge_cases():
    """Empty RPC, an empty (present) control message, empty present bytes,
    varint lengths of several bytes."""
    cases = [wire.RPC(), wire.RPC(control=wire.ControlMessage()),
             wire.RPC(publish=[wire.Message(data=b"")]),
             wire.RPC(publish=[wire.Message(data=b"x" * 70000)]),
             wire.RPC(control=wire.ControlMessage(prune=[wire.ControlPrune(b"t", [], 2**63)]))]
    for r in cases:
        assert wire.marshal(r) == to_pb(r).SerializeToString()
    assert wire.marshal(wire.RPC(control=wire.ControlMessage())) == b"\x1a\x00"


def frags_pb(rpcs):
    return [x.SerializeToString() for x in rpcs]


def test_fragment_matches_restatement_random():
    rng = np.random.default_rng(2)
    for k in range(300):
        r = rand_rpc(rng, scale=1.0 + (k % 9))
        limit = int(rng.integers(64, 3000))
        if k % 5:                                   # mostly limits every message fits under
            limit += max([to_pb(wire.RPC(publish=[m])).publish[0].ByteSize() for m in r.publish] + [0])
        try:
            want = frags_pb(wo.fragment_rpc(to_pb(r), limit))
        except wo.FragmentError:
            with pytest.raises(wire.WireError):
                wire.fragment_rpc(r, limit)
            continue
        assert wire.fragment_rpc(r, limit) == want, (k, limit)


def _mk_msg(rng, size):
    """mkMsg (gossipsub_test.go:2344-2349): data of size-4 random bytes."""
    return wire.Message(data=rng.bytes(size - 4))


@pytest.mark.parametrize("impl", ["library", "restatement"])
def test_fragment_rpc_function(impl):
    """TestFragmentRPCFunction (gossipsub_test.go:2338-2500), restated."""
    C = wo.pb()
    rng = np.random.default_rng(3)
    limit = 1024
    topic = b"test"

    def frag(r):
        if impl == "library":
            return [C["RPC"].FromString(b) for b in wire.fragment_rpc(r, limit)]
        return wo.fragment_rpc(to_pb(r), limit)

    def below(results):
        for x in results:
            assert x.ByteSize() <= limit

    r = wire.RPC(publish=[_mk_msg(rng, 10), _mk_msg(rng, 10)])
    assert len(frag(r)) == 1, "single RPC if input is < limit"

    r = wire.RPC(publish=[_mk_msg(rng, 10), _mk_msg(rng, limit * 2)])
    with pytest.raises((wire.WireError, wo.FragmentError)):
        frag(r)

    n_messages, msg_size = 100, 200
    r = wire.RPC(subscriptions=[wire.SubOpts(True, topic)], publish=[_mk_msg(rng, msg_size) for _ in range(n_messages)])
    results = frag(r)
    below(results)
    msgs_per_rpc = limit // msg_size
    assert len(results) == n_messages // msgs_per_rpc
    assert sum(len(x.publish) for x in results) == n_messages
    assert sum(len(x.subscriptions) for x in results) == 1

    r.control = wire.ControlMessage(graft=[wire.ControlGraft(topic)], prune=[wire.ControlPrune(topic)],
                                    ihave=[wire.ControlIHave(None, [b"foo"])], iwant=[wire.ControlIWant([b"bar"])])
    results = frag(r)
    below(results)
    assert len(results) == n_messages // msgs_per_rpc + 1
    assert results[-1].HasField("control")
    assert results[-1].control.SerializeToString() == to_pb(r).control.SerializeToString(), \
        "control unaltered when it fits in one RPC"

    n_topics, id_size, per_topic = 5, 32, 100
    ids = [[rng.bytes(id_size) for _ in range(per_topic)] for _ in range(n_topics)]
    r.control.ihave = [wire.ControlIHave(None, x) for x in ids]
    r.control.iwant = [wire.ControlIWant(x) for x in ids]
    results = frag(r)
    below(results)
    min_ctl = to_pb(r).control.ByteSize() // limit
    assert len(results) >= n_messages // msgs_per_rpc + min_ctl

    giant = rng.bytes(limit * 2)
    r = wire.RPC(control=wire.ControlMessage(iwant=[wire.ControlIWant([b"hello", giant])]))
    results = frag(r)
    assert len(results) == 1
    assert len(results[0].control.iwant) == 1
    assert results[0].control.iwant[0].messageIDs[0] == b"hello"


def test_fragmented_ihave_loses_its_topic():
    """The reference's fragmentRPC builds the split IHAVEs without TopicID
    (gossipsub.go:1288); kept."""
    C = wo.pb()
    r = wire.RPC(control=wire.ControlMessage(ihave=[wire.ControlIHave(b"topic", [bytes([k]) * 40 for k in range(80)])]))
    frs = [C["RPC"].FromString(b) for b in wire.fragment_rpc(r, 1024)]
    assert len(frs) > 1
    assert all(not ih.HasField("topicID") for f in frs for ih in f.control.ihave)
    assert [i for f in frs for ih in f.control.ihave for i in ih.messageIDs] == r.control.ihave[0].messageIDs


# ---- decoding (gsim_wire_decode / gsim_wire_frames) ----------------------------------

def from_pb(x) -> wire.RPC:
    """A protobuf-runtime RPC as the library's dataclasses."""
    def opt(m, f):
        return getattr(m, f) if m.HasField(f) else None
    r = wire.RPC()
    for s in x.subscriptions:
        r.subscriptions.append(wire.SubOpts(opt(s, "subscribe"), opt(s, "topicid")))
    for m in x.publish:
        r.publish.append(wire.Message(*(opt(m, f) for f in ("from", "data", "seqno", "topic", "signature", "key"))))
    if x.HasField("control"):
        c = wire.ControlMessage()
        for g in x.control.ihave:
            c.ihave.append(wire.ControlIHave(opt(g, "topicID"), list(g.messageIDs)))
        for g in x.control.iwant:
            c.iwant.append(wire.ControlIWant(list(g.messageIDs)))
        for g in x.control.graft:
            c.graft.append(wire.ControlGraft(opt(g, "topicID")))
        for p in x.control.prune:
            c.prune.append(wire.ControlPrune(opt(p, "topicID"),
                                             [wire.PeerInfo(opt(i, "peerID"), opt(i, "signedPeerRecord")) for i in p.peers],
                                             opt(p, "backoff")))
        r.control = c
    return r


def test_decode_round_trips_protobuf_runtime():
    """Random RPCs serialized by the protobuf runtime decode to the same
    fields as the runtime's own parse, and re-encode to the same bytes."""
    rng = np.random.default_rng(11)
    for k in range(400):
        r = rand_rpc(rng, scale=1.0 + (k % 7))
        data = to_pb(r).SerializeToString()
        got = wire.unmarshal(data)
        assert got == from_pb(wo.pb()["RPC"].FromString(data)), k
        assert got == r, k
        assert wire.marshal(got) == data, k


def test_decode_merges_as_proto2():
    """Concatenated encodings are one message (proto2 merge, what gogo's
    generated Unmarshal does): repeated fields append, the control message
    merges its lists, optional scalars take the last value.  The protobuf
    runtime's MergeFromString is the reference."""
    C = wo.pb()
    rng = np.random.default_rng(12)
    for k in range(200):
        parts = [to_pb(rand_rpc(rng, scale=1.0 + (k % 3))).SerializeToString() for _ in range(int(rng.integers(2, 5)))]
        want = C["RPC"]()
        for b in parts:
            want.MergeFromString(b)
        got = wire.unmarshal(b"".join(parts))
        assert got == from_pb(want), k
        assert wire.marshal(got) == want.SerializeToString(), k


def test_decode_skips_unknown_fields():
    """Fields the schema does not know (every wire type, nested groups)
    are skipped at every level, as gogo's skipRpc does."""
    C = wo.pb()
    rng = np.random.default_rng(13)
    unknown = [b"\x78\x05",                          # field 15, varint
               b"\x81\x01" + bytes(8),                # field 16, fixed64
               b"\x8d\x01" + bytes(4),                # field 17, fixed32
               b"\x92\x01\x03abc",                   # field 18, bytes
               b"\x9b\x01\x08\x01\xa3\x01\xa4\x01\x9c\x01"]   # field 19, a group holding a group
    for k in range(100):
        r = rand_rpc(rng)
        data = to_pb(r).SerializeToString()
        junk = b"".join(unknown[int(q)] for q in rng.integers(0, len(unknown), size=3))
        got = wire.unmarshal(junk + data + junk)
        assert got == r, k
        want = C["RPC"]()
        want.MergeFromString(junk + data + junk)
        want.DiscardUnknownFields()
        assert wire.marshal(got) == want.SerializeToString()
    # inside the nested messages too: a PRUNE's PeerInfo with an unknown field
    pi = b"\x0a\x02id" + unknown[3] + b"\x12\x01r"
    prune = b"\x0a\x01t" + b"\x12" + bytes([len(pi)]) + pi + b"\x18\x3c"
    ctl = b"\x22" + bytes([len(prune)]) + prune
    got = wire.unmarshal(b"\x1a" + bytes([len(ctl)]) + ctl)
    assert got.control.prune == [wire.ControlPrune(b"t", [wire.PeerInfo(b"id", b"r")], 60)]


def test_decode_rejects_malformed():
    """What gogo's Unmarshal errors on (a "bogus rpc", comm.go:82)."""
    good = wire.marshal(wire.RPC(subscriptions=[wire.SubOpts(True, b"t")],
                                 publish=[wire.Message(data=b"hello", seqno=bytes(8))],
                                 control=wire.ControlMessage(graft=[wire.ControlGraft(b"t")])))
    for cut in range(1, len(good)):          # truncated inside a field
        try:
            wire.unmarshal(good[:cut])
        except wire.WireError:
            continue
        # a cut at a field boundary of the top level is a valid shorter RPC
        assert wire.marshal(wire.unmarshal(good[:cut])) == good[:cut]
    bad = [b"\x0a\x05\x08",                       # length past the end
           b"\x08\x01",                            # RPC.subscriptions with a varint wire type
           b"\x0a\x02\x0a\x00",                    # SubOpts.subscribe with a bytes wire type
           b"\x1a\x03\x22\x01\x18",                 # ControlPrune.backoff cut
           b"\x00\x00",                            # field number 0
           b"\x0c",                                 # end group with none open
           b"\x78" + b"\xff" * 10 + b"\x01",        # varint over 64 bits
           b"\x7e\x00"]                             # wire type 6
    for b in bad:
        with pytest.raises(wire.WireError):
            wire.unmarshal(b)
    assert wire.unmarshal(b"") == wire.RPC()
    assert wire.unmarshal(b"\x1a\x00") == wire.RPC(control=wire.ControlMessage())


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def test_decode_field_numbers_as_generated_code():
    """Tag handling of gogo's generated Unmarshal (pb/rpc.pb.go:1345-1352):
    fieldNum := int32(wire >> 3), rejected only when <= 0, so a large number
    is an unknown field, one of 2^31 or more is illegal, and 2^32 + f wraps
    to field f; skipRpc (rpc.pb.go:2566-2641) takes any field number inside
    a group, field 0 included."""
    sub = wire.marshal(wire.RPC(subscriptions=[wire.SubOpts(True, b"t")]))   # field 1, bytes
    want = wire.unmarshal(sub)
    body = sub[2:]
    for fn in (0x20000000, 0x7FFFFFFF):               # unknown, above the old 29-bit cap
        assert wire.unmarshal(_varint(fn << 3) + b"\x05" + sub) == want, fn
    for fn in (0x80000000, 0xFFFFFFFF):               # int32 <= 0: illegal tag
        with pytest.raises(wire.WireError):
            wire.unmarshal(_varint(fn << 3) + b"\x05" + sub)
    wrapped = _varint(((1 << 32) + 1) << 3 | 2) + bytes([len(body)]) + body   # field 2^32 + 1 = subscriptions
    assert wire.unmarshal(wrapped) == want
    group0 = b"\x9b\x01" + b"\x00\x05" + b"\x9c\x01"   # field 19 group holding field 0
    assert wire.unmarshal(group0 + sub) == want


def test_decode_fragments_of_fragment_rpc_function():
    """The fragments TestFragmentRPCFunction's RPCs split into
    (gossipsub_test.go:2338-2500) decode to the original's contents, in
    order: messages, subscriptions, grafts, prunes, iwant and ihave ids."""
    rng = np.random.default_rng(14)
    topic = b"test"
    ids = [[rng.bytes(32) for _ in range(100)] for _ in range(5)]
    r = wire.RPC(subscriptions=[wire.SubOpts(True, topic)], publish=[_mk_msg(rng, 200) for _ in range(100)],
                 control=wire.ControlMessage(graft=[wire.ControlGraft(topic)], prune=[wire.ControlPrune(topic)],
                                             ihave=[wire.ControlIHave(None, x) for x in ids],
                                             iwant=[wire.ControlIWant(x) for x in ids]))
    frs = [wire.unmarshal(b) for b in wire.fragment_rpc(r, 1024)]
    assert [m for f in frs for m in f.publish] == r.publish
    assert [x for f in frs for x in f.subscriptions] == r.subscriptions
    ctl = [f.control for f in frs if f.control is not None]
    assert [g for c in ctl for g in c.graft] == r.control.graft
    assert [p for c in ctl for p in c.prune] == r.control.prune
    assert [i for c in ctl for g in c.iwant for i in g.messageIDs] == [i for x in ids for i in x]
    assert [i for c in ctl for g in c.ihave for i in g.messageIDs] == [i for x in ids for i in x]


def test_frames_split_a_delimited_stream():
    """msgio's varint-delimited reader (comm.go:64-82): whole frames, a
    partial one left for later, frames over maxMessageSize refused."""
    rng = np.random.default_rng(15)
    rpcs = [to_pb(rand_rpc(rng, scale=1 + k % 5)).SerializeToString() for k in range(30)] + [b"", b"x" * 300]
    stream = wire.delimited(rpcs)
    got, used = wire.frames(stream)
    assert got == rpcs and used == len(stream)
    assert [wire.unmarshal(b) for b in got[:30]] == [wire.unmarshal(b) for b in rpcs[:30]]
    for cut in (1, len(stream) // 3, len(stream) - 1):
        part, used = wire.frames(stream[:cut])
        assert part == rpcs[:len(part)] and stream[:used] == wire.delimited(part)
        rest, _ = wire.frames(stream[used:])
        assert part + rest == rpcs
    with pytest.raises(wire.WireError):
        wire.frames(wire.delimited([b"y" * 2000]), max_size=1024)
    ok, _ = wire.frames(wire.delimited([b"y" * 1024]), max_size=1024)
    assert ok == [b"y" * 1024]


# ---- GPU ----------------------------------------------------------------------------


def expected_heartbeat_rpcs(net, st, msgs, mcaches, lib, T, names, backoff, p0, p1, peer_ids=None, px=None,
                            unsub_backoff=None):
    """CPU build of the heartbeat RPCs of senders [p0, p1): GRAFT/PRUNE from
    the oracle's inbox (parity 0, the receiver's edge), IHAVE from its
    emitGossip marks, ids from the pinned mcaches (GetGossipIDs order).
    px: {(pruner, pruned, topic): [listed peers]} -- the PX lists the oracle's
    makePrune chose (ORC_EV_PX_PEER); a Leave's PRUNE (CTL_UNSUB) carries
    unsub_backoff."""
    import ctypes
    C = wo.pb()
    E = net.e
    marks = msgs.ihave_marks(E)
    rev = st.rev
    buf = (ctypes.c_uint64 * 65536)()
    out = []
    for p in range(p0, p1):
        gids = {}
        for e in range(int(net.row_ptr[p]), int(net.row_ptr[p + 1])):
            q = int(net.col[e])
            re = int(rev[e])
            r = C["RPC"]()
            c = r.control
            any_ = False
            for t in range(T):
                if marks[t, re]:
                    if t not in gids:
                        k = lib.orc_mcache_gossip_ids(mcaches[p], t, buf, 65536)
                        gids[t] = [int(buf[i]) for i in range(k)]
                    ids = []
                    for mid in gids[t]:
                        pre = b"" if peer_ids is None else bytes(peer_ids[int(msgs.origin[mid % msgs.seen.shape[0]])])
                        ids.append(pre + int(mid).to_bytes(8, "big"))
                    c.ihave.add(topicID=names[t], messageIDs=ids)
                    any_ = True
            for t in range(T):
                if st.ctl[0, t, re] & 0x01:
                    c.graft.add(topicID=names[t])
                    any_ = True
            for t in range(T):
                ct = int(st.ctl[0, t, re])
                if ct & 0x02:
                    x = c.prune.add(topicID=names[t])
                    if ct & _abi.CTL_PX:
                        for y in (px or {}).get((p, q, t), []):
                            x.peers.add(peerID=bytes(peer_ids[y]) if peer_ids is not None else int(y).to_bytes(4, "big"))
                    x.backoff = unsub_backoff if (ct & _abi.CTL_UNSUB) else backoff
                    any_ = True
            if any_:
                out.append((p, q, r.SerializeToString()))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("with_peer_ids,px", [(False, False), (True, False), (False, True), (True, True)])
def test_heartbeat_rpcs_match_oracle(require_gpu, with_peer_ids, px):
    """px: WithPeerExchange, meshes above Dhi (the heartbeat prunes with PX)
    and Leaves (their PRUNEs carry PX too, UnsubscribeBackoff): every PRUNE's
    PeerInfo list equals the oracle's makePrune choice."""
    import oracle_binding as ob
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from gsim.params import GossipSubParams, PeerScoreThresholds, Second
    from test_heartbeat import tick_time
    from tickrun import run_parity, subscribed_schedule
    n, k, T = 600, 12, 3
    rng = np.random.default_rng(91)
    params = beacon_params(T)
    gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2, PeerExchange=px)
    th = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-100, GraylistThreshold=-300)
    net = random_regular(n, k, seed=n + 1, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), (11 if px else 6) / k)
    ticks = list(range(1, 7))
    sched = subscribed_schedule(rng, ticks, net, T, 5.0, 0.0, verdicts=(0.85, 0.05, 0.05, 0.05, 0.0))
    subs = None
    if px:                                  # Leaves at ticks 3 and 5 (PRUNE | UNSUB | PX)
        subs = {kk: [(np.array([(int(p), int(rng.integers(0, T))) for p in rng.choice(n, 25, replace=False)],
                               dtype=np.uint32), False)] for kk in (3, 5)}
    names = [f"topic{t:02d}".encode() for t in range(T)]
    peer_ids = rng.integers(0, 256, size=(n, 38), dtype=np.uint8) if with_peer_ids else None
    lib = ob.load()
    backoff = int(gp.PruneBackoff // Second)
    unsub_backoff = int(gp.UnsubscribeBackoff // Second)
    state = {"mc": None, "checked": 0, "px": 0, "px_leave": 0}

    def after_heartbeat(kk, eng, st_, msgs):
        if state["mc"] is None:
            msgs.log()                      # the Put stream starts now: windows are empty before tick 1
            state["mc"] = [lib.orc_mcache_new(gp.HistoryGossip, gp.HistoryLength) for _ in range(n)]
        mc = state["mc"]
        ev = msgs.events()
        lists = {}
        for e in ev:
            if int(e["kind"]) == ob.EV_PUT:
                lib.orc_mcache_put(mc[int(e["a"])], int(e["mid"]), int(e["topic"]))
            # this tick's makePrune lists: the heartbeat's and the Leaves' before it (not the
            # last tick's GRAFT replies)
            if int(e["kind"]) == ob.EV_PX_PEER and int(e["x"]) in (tick_time(kk), tick_time(kk) - Second // 2):
                lists.setdefault((int(e["a"]), int(e["mid"]), int(e["topic"])), []).append((int(e["g"]), int(e["b"])))
        px_lists = {key: [y for _, y in sorted(v)] for key, v in lists.items()}
        if kk >= 2:
            p0, p1 = 37, 337
            got = wire.heartbeat_rpcs(eng, kk, p0, p1, names, peer_ids=peer_ids, prune_backoff_s=backoff)
            want = expected_heartbeat_rpcs(net, st_, msgs, mc, lib, T, names, backoff, p0, p1, peer_ids, px=px_lists,
                                           unsub_backoff=unsub_backoff)
            for (_, _, b_) in want:
                r_ = wo.pb()["RPC"].FromString(b_)
                state["px"] += sum(len(x.peers) > 0 for x in r_.control.prune)
                state["px_leave"] += sum(len(x.peers) > 0 and x.backoff == unsub_backoff for x in r_.control.prune)
            assert len(got) == len(want), f"tick {kk}: {len(got)} RPCs, expected {len(want)}"
            for g_, w_ in zip(got, want):
                assert g_ == w_, f"tick {kk}: RPC {g_[0]}->{g_[1]} differs"
            state["checked"] += len(got)
            # their SendRPC / RecvRPC trace events (trace.go:250-324, traceRPCMeta 326-414)
            pid = (lambda p: bytes(peer_ids[p])) if peer_ids is not None else (lambda p: int(p).to_bytes(4, "big"))
            assert wire.trace_rpc_batch(got, names, peer_ids=peer_ids, timestamp=tick_time(kk), which=3) == \
                wo.trace_rpc_events(want, pid, tick_time(kk), 3), f"tick {kk}: RPC trace events differ"
        for p in range(n):                  # the heartbeat ends with mcache.Shift
            lib.orc_mcache_shift(mc[p])

    try:
        run_parity(net, params, th, gp, st, ticks, sched, ring=512, after_heartbeat=after_heartbeat, subs=subs)
    finally:
        for m in state["mc"] or []:
            lib.orc_mcache_free(m)
    assert state["checked"] > 200
    if px:
        assert state["px"] > 20 and state["px_leave"] > 0, state


@pytest.mark.gpu
def test_heartbeat_rpcs_refuse_what_they_cannot_encode(require_gpu):
    """A heartbeat output the device encoder does not hold per RPC is
    refused rather than encoded wrongly: emitGossip's per-target random
    MaxIHaveLength-subsets (gossipsub.go:1763-1772: a window longer than
    MaxIHaveLength).  (makePrune's PX lists are encoded:
    test_heartbeat_rpcs_match_oracle[px].)"""
    import oracle_binding as ob
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from gsim.params import GossipSubParams, PeerScoreThresholds, Second
    from test_heartbeat import tick_time
    from tickrun import run_parity, subscribed_schedule
    n, k, T = 400, 16, 2
    names = [f"t{t}".encode() for t in range(T)]
    th = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-100, GraylistThreshold=-300)
    params = beacon_params(T)
    for case in ("window",):
        rng = np.random.default_rng(7)
        if case == "window":
            gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2, MaxIHaveLength=2)
            rate, p_mesh = 8.0, 6 / k
        else:
            gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2, PeerExchange=True)
            rate, p_mesh = 2.0, 14 / k          # meshes above Dhi: the heartbeat prunes with PX
        net = random_regular(n, k, seed=33, n_topics=T)
        st = ob.NetState(net, params, thresholds=th, gossip=gp)
        synthetic_state(st, rng, tick_time(0), p_mesh)
        ticks = [1, 2, 3]
        sched = subscribed_schedule(rng, ticks, net, T, rate, 0.0)
        seen = {"refused": 0, "encoded": 0}

        def after_heartbeat(kk, eng, st_, msgs):
            # the oracle's inbox says which PRUNEs carry PX (GSIM_CTL_PX, parity 0)
            refuse = kk >= 2 if case == "window" else bool(((st_.ctl[0] & 0x04) != 0).any())
            if not refuse:
                wire.heartbeat_rpcs(eng, kk, 0, n, names, prune_backoff_s=int(gp.PruneBackoff // Second))
                seen["encoded"] += 1
                return
            with pytest.raises(wire.WireError) as ex:
                wire.heartbeat_rpcs(eng, kk, 0, n, names, prune_backoff_s=int(gp.PruneBackoff // Second))
            msg = str(ex.value)
            assert ("MaxIHaveLength" in msg) if case == "window" else ("peer exchange" in msg), msg
            seen["refused"] += 1

        run_parity(net, params, th, gp, st, ticks, sched, ring=256, after_heartbeat=after_heartbeat)
        assert seen["refused"] >= 1 and seen["encoded"] >= 1, (case, seen)
