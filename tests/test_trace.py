"""Trace export: the pubsubTracer events
(trace.go:70-530) of a range of routers, and their TraceEventBatch encoding
(pb/trace.proto).

CPU part:
  * gsim_trace_encode is byte-identical to the protobuf runtime's serializer
    on a restatement of pb/trace.proto (oracle/wire_oracle.py trace_pb) for
    every event type the engine produces;
  * the oracle's event log, read as a trace, keeps the tracer's rules: one
    DELIVER or REJECT per (router, message) at its first reception, later
    copies DUPLICATE, a PUBLISH at the origin.
GPU part: the engine's trace of routers [lo, hi) equals the oracle's log
event for event (time, router, type, peer, topic, message, reason) after
every tick of a network with gossip, every validation verdict, mesh churn
and connection churn."""
import os
import sys

import numpy as np
import pytest

import oracle_binding as ob
from conftest import REPO
from gsim import _abi, wire
from gsim.engine import Engine
from gsim.params import GossipSubParams, PeerScoreThresholds, Second

sys.path.insert(0, os.path.join(REPO, "oracle"))
import wire_oracle as wo  # noqa: E402  (test infrastructure)

from test_delivery import R, T0  # noqa: E402
from test_heartbeat import SEED, tick_time  # noqa: E402

REASONS = {1: "validation failed", 2: "validation ignored", 3: "validation throttled", 4: "invalid signature"}


def _pid(p, peer_ids):
    return bytes(peer_ids[p]) if peer_ids is not None else int(p).to_bytes(4, "big")


def _rpc_units(recs):
    """The TraceEvents of the records: an IWANT answer's messages (RPC
    records of reason 1 with the same time, router, type and peer, adjacent
    in gsim_trace_read's order) are one RPC, every other record one event."""
    out, k = [], 0
    while k < len(recs):
        q = k + 1
        r = recs[k]
        if int(r["type"]) in (_abi.TRACE_RECV_RPC, _abi.TRACE_SEND_RPC) and int(r["reason"]) in (1, 2):
            while q < len(recs) and all(recs[q][f] == r[f] for f in ("type", "reason", "timestamp", "peer", "other")):
                q += 1
        out.append(recs[k:q])
        k = q
    return out


def _expected_batch(recs, names, peer_ids, proto=b"/meshsub/1.1.0"):
    C = wo.trace_pb()
    batch = C["TraceEventBatch"]()
    for unit in _rpc_units(recs):
        r = unit[0]
        e = batch.batch.add()
        typ = int(r["type"])
        e.type = typ
        e.peerID = _pid(int(r["peer"]), peer_ids)
        e.timestamp = int(r["timestamp"])
        mid = int(r["msg_id"]).to_bytes(8, "big")
        other = _pid(int(r["other"]), peer_ids)
        topic = names[int(r["topic"])].decode() if int(r["topic"]) >= 0 else None
        if typ in (_abi.TRACE_RECV_RPC, _abi.TRACE_SEND_RPC):
            # RecvRPC{receivedFrom, meta} / SendRPC{sendTo, meta}, RPCMeta.messages (trace.go:250-345)
            x = e.recvRPC if typ == _abi.TRACE_RECV_RPC else e.sendRPC
            if typ == _abi.TRACE_RECV_RPC:
                x.receivedFrom = other
            else:
                x.sendTo = other
            if int(r["reason"]) == 2:
                # an IWANT request: RPCMeta.control.iwant = [ControlIWantMeta{messageIDs}]
                x.meta.control.iwant.add().messageIDs.extend(int(y["msg_id"]).to_bytes(8, "big") for y in unit)
                continue
            for y in unit:
                mm = x.meta.messages.add()
                mm.messageID = int(y["msg_id"]).to_bytes(8, "big")
                mm.topic = names[int(y["topic"])].decode()
            continue
        if typ == _abi.TRACE_PUBLISH_MESSAGE:
            e.publishMessage.messageID, e.publishMessage.topic = mid, topic
        elif typ == _abi.TRACE_REJECT_MESSAGE:
            x = e.rejectMessage
            x.messageID, x.receivedFrom, x.reason, x.topic = mid, other, REASONS[int(r["reason"])], topic
        elif typ == _abi.TRACE_DUPLICATE_MESSAGE:
            x = e.duplicateMessage
            x.messageID, x.receivedFrom, x.topic = mid, other, topic
        elif typ == _abi.TRACE_DELIVER_MESSAGE:
            x = e.deliverMessage
            x.messageID, x.topic, x.receivedFrom = mid, topic, other
        elif typ == _abi.TRACE_ADD_PEER:
            e.addPeer.peerID, e.addPeer.proto = other, proto.decode()
        elif typ == _abi.TRACE_REMOVE_PEER:
            e.removePeer.peerID = other
        elif typ == _abi.TRACE_GRAFT:
            e.graft.peerID, e.graft.topic = other, topic
        elif typ == _abi.TRACE_PRUNE:
            e.prune.peerID, e.prune.topic = other, topic
        elif typ == _abi.TRACE_JOIN:
            e.join.topic = topic
        elif typ == _abi.TRACE_LEAVE:
            e.leave.topic = topic
    return batch.SerializeToString()


def _random_records(rng, n, T, N):
    types = [0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11, 12]
    recs = np.zeros(n, dtype=Engine.TRACE_DTYPE)
    for k in range(n):
        typ = types[rng.integers(0, len(types))]
        recs[k]["type"] = typ
        recs[k]["timestamp"] = int(rng.integers(-5, 1 << 62))
        recs[k]["peer"] = rng.integers(0, N)
        recs[k]["other"] = rng.integers(0, N)
        recs[k]["msg_id"] = int(rng.integers(0, 1 << 63))
        recs[k]["topic"] = -1 if typ in (4, 5) else rng.integers(0, T)
        recs[k]["reason"] = rng.integers(1, 5) if typ == 1 else rng.integers(0, 3) if typ in (6, 7) else 0
        if typ in (6, 7) and recs[k]["reason"] in (1, 2) and k > 0 and rng.random() < 0.6:
            # another message of the same IWANT answer / another id of the same IWANT request
            for f in ("type", "timestamp", "peer", "other"):
                recs[k][f] = recs[k - 1][f] if recs[k - 1]["type"] == typ else recs[k][f]
            if recs[k - 1]["type"] == typ and recs[k - 1]["reason"] in (1, 2):
                recs[k]["reason"] = recs[k - 1]["reason"]
    return recs


def test_pb_tracer_stream():
    """PBTracer's file (tracer.go:130-179, protoio's DelimitedWriter): every
    TraceEvent of the batch, varint-delimited, in order."""
    C = wo.trace_pb()
    rng = np.random.default_rng(29)
    names = [f"t{t}".encode() for t in range(3)]
    recs = _random_records(rng, 150, 3, 200)
    batch = wire.trace_batch(recs, names)
    frames, used = wire.frames(wire.pb_tracer_stream(batch))
    want = C["TraceEventBatch"].FromString(batch).batch
    assert used == len(wire.pb_tracer_stream(batch)) and len(frames) == len(want) > 0
    for f, w in zip(frames, want):
        assert C["TraceEvent"].FromString(f) == w
    assert wire.pb_tracer_stream(b"") == b""
    with pytest.raises(wire.WireError):
        wire.pb_tracer_stream(b"\x08\x01")


@pytest.mark.parametrize("with_ids", [False, True])
def test_trace_encode_matches_protobuf_runtime(with_ids):
    rng = np.random.default_rng(17 + with_ids)
    T, N = 5, 300
    names = [f"/eth2/topic/{t:03d}".encode() for t in range(T)]
    peer_ids = rng.integers(0, 256, size=(N, 38), dtype=np.uint8) if with_ids else None
    for n in (0, 1, 7, 200):
        recs = _random_records(rng, n, T, N)
        got = wire.trace_batch(recs, names, peer_ids=peer_ids)
        assert got == _expected_batch(recs, names, peer_ids)


def test_oracle_log_follows_tracer_rules():
    """Read as a trace: a router's first reception of a message is one
    DELIVER (accepted) or REJECT (with the verdict as reason), every later
    copy a DUPLICATE; bad-signature copies are REJECT each; the origin
    publishes."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import oracle_trace, subscribed_schedule
    rng = np.random.default_rng(23)
    n, k, T = 500, 16, 2
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-2000, PublishThreshold=-4000, GraylistThreshold=-8000)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    net = random_regular(n, k, seed=31, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    ticks = list(range(1, 5))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.0, verdicts=(0.6, 0.1, 0.1, 0.1, 0.1))
    msgs = ob.Msgs(n, T, 256, R, T0, Second)
    msgs.log()
    lib = ob.load()
    seen_first = {}
    counts = np.zeros(13, dtype=np.int64)
    for kk in ticks:
        now = tick_time(kk)
        v = st.view()
        lib.orc_refresh_scores(v, now)
        msgs.penalties(st, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
        msgs.heartbeat(st, kk, now, SEED)
        for g in range(kk * R, kk * R + R):
            for (mid, t, o, inv) in sched.get(g, []):
                msgs.publish(st, mid, t, o, inv, g)
            msgs.round(st, g)
        tr = oracle_trace(msgs.events(), msgs, 0, n)
        counts += np.bincount(tr["type"], minlength=13)
        dups = []
        for r in tr:
            typ, key = int(r["type"]), (int(r["peer"]), int(r["msg_id"]))
            if typ in (_abi.TRACE_DELIVER_MESSAGE, _abi.TRACE_PUBLISH_MESSAGE) or \
                    (typ == _abi.TRACE_REJECT_MESSAGE and int(r["reason"]) != 4):
                assert key not in seen_first, "one first reception per router and message"
                seen_first[key] = int(r["timestamp"])
            elif typ == _abi.TRACE_DUPLICATE_MESSAGE:
                dups.append((key, int(r["timestamp"])))
        for key, ts in dups:                            # same-round copies share the timestamp
            assert key in seen_first and seen_first[key] <= ts, "a duplicate follows the first reception"
    for typ in (_abi.TRACE_PUBLISH_MESSAGE, _abi.TRACE_REJECT_MESSAGE, _abi.TRACE_DUPLICATE_MESSAGE,
                _abi.TRACE_DELIVER_MESSAGE, _abi.TRACE_GRAFT, _abi.TRACE_PRUNE):
        assert counts[typ] > 0, f"event type {typ} occurs"


@pytest.mark.gpu
@pytest.mark.parametrize("lo,hi,shards", [(0, 1000, 0), (137, 400, 0), (0, 1000, 3), (137, 400, 2)])
def test_trace_bit_exact(require_gpu, lo, hi, shards):
    """Every event type the engine produces, IWANT requests (reason 2) and
    answers (reason 1) included, equals the oracle's log; on 2 / 3 shards
    through gsim_group_trace_* (a range that starts and ends inside shards)."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import run_parity, subscribed_schedule
    rng = np.random.default_rng(99 + lo)
    n, k, T = 1000, 16, 3
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-200, PublishThreshold=-400, GraylistThreshold=-800)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    net = random_regular(n, k, seed=77, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.6)          # meshes over Dhi: heartbeat prunes
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.0, verdicts=(0.7, 0.08, 0.08, 0.07, 0.07))
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 30, replace=False)]
    churn = {2: [(down, False)], 4: [(down, True)]}
    log = []
    eng = None
    if shards:
        from gsim.shard import ShardedEngine
        eng = ShardedEngine(params, th, gossip=gp, shards=shards)
        eng.load_graph(net)
        eng.set_seed(SEED)
        st.push_to_engine(eng)
    run_parity(net, params, th, gp, st, ticks, sched, ring=512, churn=churn, trace=(lo, hi), trace_log=log, eng=eng)
    total = np.sum([x[0] for x in log], axis=0)
    for typ in (0, 1, 2, 3, 4, 5, 6, 7, 11, 12):
        assert total[typ] > 0, f"event type {typ} traced"
    reasons = np.sum([x[1] for x in log], axis=0)
    assert reasons[1] > 0 and reasons[2] > 0, "IWANT answers and requests traced"


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [0, 2])
def test_trace_read_every_round_bit_exact(require_gpu, shards):
    """The trace read after every round: an IWANT request of control round 0
    is stamped at round 1, so a read right after round 0 keeps it, already
    resolved, for the next read; that read must not resolve it again (its id
    is a wire id by then).  The tick's reads together equal the oracle's log,
    on one engine and on 2 shards."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import run_parity, subscribed_schedule
    rng = np.random.default_rng(404)
    n, k, T = 600, 16, 2
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-200, PublishThreshold=-400, GraylistThreshold=-800)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    net = random_regular(n, k, seed=78, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.6)
    ticks = list(range(1, 4))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.0, verdicts=(0.8, 0.05, 0.05, 0.05, 0.05))
    log = []
    eng = None
    if shards:
        from gsim.shard import ShardedEngine
        eng = ShardedEngine(params, th, gossip=gp, shards=shards)
        eng.load_graph(net)
        eng.set_seed(SEED)
        st.push_to_engine(eng)
    run_parity(net, params, th, gp, st, ticks, sched, ring=256, trace=(0, n), trace_log=log, eng=eng,
               trace_every_round=True)
    reasons = np.sum([x[1] for x in log], axis=0)
    assert reasons[2] > 0, "IWANT requests traced (the events kept across reads)"


def _random_rpc(rng, P):
    """An RPC with every part traceRPCMeta reads, optional fields present or
    absent at random (pb() classes)."""
    rpc = P["RPC"]()
    for _ in range(rng.integers(0, 3)):
        s = rpc.subscriptions.add()
        if rng.random() < 0.7:
            s.subscribe = bool(rng.integers(0, 2))
        if rng.random() < 0.8:
            s.topicid = f"t{rng.integers(0, 9)}".encode()
    for _ in range(rng.integers(0, 3)):
        m = rpc.publish.add()
        setattr(m, "from", bytes(rng.integers(0, 256, size=6, dtype=np.uint8)))
        m.seqno = int(rng.integers(0, 2**63)).to_bytes(8, "big")
        m.data = b"x" * int(rng.integers(0, 5))
        if rng.random() < 0.8:
            m.topic = f"topic-{rng.integers(0, 5)}".encode()
    if rng.random() < 0.85:
        c = rpc.control
        c.SetInParent()
        for _ in range(rng.integers(0, 3)):
            ih = c.ihave.add()
            if rng.random() < 0.8:
                ih.topicID = b"ih" + bytes([97 + int(rng.integers(0, 5))])
            ih.messageIDs.extend(bytes(rng.integers(0, 256, size=10, dtype=np.uint8))
                                 for _ in range(rng.integers(0, 4)))
        for _ in range(rng.integers(0, 2)):
            c.iwant.add().messageIDs.extend(bytes(rng.integers(0, 256, size=7, dtype=np.uint8))
                                            for _ in range(rng.integers(0, 3)))
        for _ in range(rng.integers(0, 3)):
            g = c.graft.add()
            if rng.random() < 0.8:
                g.topicID = b"gr"
        for _ in range(rng.integers(0, 3)):
            pr = c.prune.add()
            if rng.random() < 0.8:
                pr.topicID = b"pr"
            pr.backoff = int(rng.integers(0, 100))
            for _ in range(rng.integers(0, 3)):
                pi = pr.peers.add()
                if rng.random() < 0.8:
                    pi.peerID = bytes(rng.integers(0, 256, size=5, dtype=np.uint8))
                if rng.random() < 0.3:
                    pi.signedPeerRecord = b"rec"
    return rpc


@pytest.mark.parametrize("with_ids,which", [(False, 3), (True, 7), (True, 1)])
def test_rpc_trace_events_match_trace_rpc_meta(with_ids, which):
    """gsim_trace_rpc_encode against traceRPCMeta restated on the protobuf
    runtime (oracle/wire_oracle.py): SendRPC / RecvRPC / DropRPC events of
    RPCs with subscriptions, published messages, IHAVE / IWANT / GRAFT / PRUNE
    (with and without PX peers and optional fields), and empty control."""
    rng = np.random.default_rng(31 + which)
    P = wo.pb()
    N = 50
    peer_ids = rng.integers(0, 256, size=(N, 38), dtype=np.uint8) if with_ids else None
    rpcs = []
    for _ in range(60):
        a, b = (int(x) for x in rng.integers(0, N, size=2))
        rpcs.append((a, b, _random_rpc(rng, P).SerializeToString()))
    pid = (lambda p: bytes(peer_ids[p])) if with_ids else (lambda p: int(p).to_bytes(4, "big"))
    ts = 1_700_000_000_123_456_789
    got = wire.trace_rpc_batch(rpcs, peer_ids=peer_ids, timestamp=ts, which=which)
    assert got == wo.trace_rpc_events(rpcs, pid, ts, which)
    T = wo.trace_pb()
    batch = T["TraceEventBatch"]()
    batch.ParseFromString(got)
    assert len(batch.batch) == len(rpcs) * bin(which).count("1")
    with pytest.raises(wire.WireError):
        wire.trace_rpc_batch([(0, 1, b"\x0a\x05ab")], which=1)        # truncated field


def test_trace_encode_rejects_unknown_types_and_short_buffers():
    import ctypes
    names = [b"t0"]
    recs = np.zeros(1, dtype=Engine.TRACE_DTYPE)
    recs[0]["type"] = 8                    # DROP_RPC: not produced by the engine
    with pytest.raises(wire.WireError):
        wire.trace_batch(recs, names)
    recs[0]["type"] = 6                    # RECV_RPC without a topic: malformed
    recs[0]["topic"] = -1
    with pytest.raises(wire.WireError):
        wire.trace_batch(recs, names)
    recs[0]["topic"] = 0
    recs[0]["type"] = _abi.TRACE_REMOVE_PEER
    lib = _abi.load()
    nm = _abi.CWireNames()
    tn = (_abi.CBytes * 1)()
    buf = ctypes.create_string_buffer(b"t0", 2)
    tn[0] = _abi.CBytes(ctypes.addressof(buf), 2)
    nm.topic_names = ctypes.addressof(tn)
    n = ctypes.c_uint64()
    out = ctypes.create_string_buffer(4)
    rc = lib.gsim_trace_encode(recs.ctypes.data_as(ctypes.c_void_p), 1, ctypes.byref(nm), b"p", out, 4,
                               ctypes.byref(n))
    assert rc == _abi.GSIM_ERANGE and n.value == len(wire.trace_batch(recs, names))
