"""Lock-step runner: the engine (HIP, through the C ABI) and the oracle (C)
advance the same network tick by tick — refresh + P7 penalties + scores,
heartbeat with emitGossip, R propagation rounds with publications, optional
churn between ticks — and every observable array is compared bit-for-bit
after each tick.  Shared by the per-configuration parity tests."""
import numpy as np

import oracle_binding as ob
from gsim import _abi
from gsim.params import Second
from test_delivery import R, T0
from test_heartbeat import SEED, assert_same, tick_time


def restrict_to_subscriptions(st, net):
    """Zero the topic state of every (topic, edge) whose endpoints do not
    share the topic: no mesh link and no topicStats can exist there."""
    owner = net.owner()
    for t in range(st.T):
        bit = np.uint64(1 << t)
        shared = ((net.sub[owner] & bit) != 0) & ((net.sub[net.col] & bit) != 0)
        off = ~shared
        for f in ("first", "meshd", "fail", "invalid"):
            getattr(st, f)[t, off] = 0.0
        st.graft_time[t, off] = 0
        st.mesh_time[t, off] = 0
        st.tflags[t, off] = 0


def oracle_trace(ev, msgs, lo, hi):
    """The oracle's event log as the engine's trace records (gsim_trace_event)
    of the routers [lo, hi), sorted as gsim_trace_read sorts them."""
    from gsim.engine import Engine
    out = []
    ring = msgs.seen.shape[0]
    for e in ev:
        kind, a, b = int(e["kind"]), int(e["a"]), int(e["b"])
        mid, topic = int(e["mid"]), int(e["topic"])
        if kind == ob.EV_RPC_MSG:
            # a message RPC: SEND_RPC at the sender, RECV_RPC at the receiver; an IWANT
            # answer (x = 1) is sent the round before it arrives
            g, x = int(e["g"]), int(e["x"])
            if lo <= a < hi:
                out.append((msgs.round_time(g - x), mid, a, b, topic, _abi.TRACE_SEND_RPC, x))
            if lo <= b < hi:
                out.append((msgs.round_time(g), mid, b, a, topic, _abi.TRACE_RECV_RPC, x))
            continue
        if kind == ob.EV_RPC_IWANT:
            # handleIHave's IWANT (reason 2): sent in control round g, handled in g + 1
            g = int(e["g"])
            if lo <= a < hi:
                out.append((msgs.round_time(g), mid, a, b, topic, _abi.TRACE_SEND_RPC, 2))
            if lo <= b < hi:
                out.append((msgs.round_time(g + 1), mid, b, a, topic, _abi.TRACE_RECV_RPC, 2))
            continue
        if not (lo <= a < hi):
            continue
        if kind == ob.EV_PUBLISH:
            out.append((msgs.round_time(int(e["g"])), mid, a, a, topic, _abi.TRACE_PUBLISH_MESSAGE, 0))
        elif kind == ob.EV_SEEN and b != 0xFFFFFFFF:
            ts = msgs.round_time(int(e["g"]))
            if int(e["x"]):
                # the slot holding the message (sub-rings: not id % ring)
                slots = np.nonzero(msgs.mid == np.uint64(mid))[0]
                vd = int(msgs.invalid[slots[0] if len(slots) else mid % ring])
                typ = _abi.TRACE_DELIVER_MESSAGE if vd == 0 else _abi.TRACE_REJECT_MESSAGE
                out.append((ts, mid, a, b, topic, typ, vd))
            else:
                out.append((ts, mid, a, b, topic, _abi.TRACE_DUPLICATE_MESSAGE, 0))
        elif kind == ob.EV_REJECT_SIG:
            out.append((msgs.round_time(int(e["g"])), mid, a, b, topic, _abi.TRACE_REJECT_MESSAGE, 4))
        elif kind in (ob.EV_GRAFT, ob.EV_PRUNE, ob.EV_ADD_PEER, ob.EV_REMOVE_PEER, ob.EV_JOIN, ob.EV_LEAVE):
            typ = {ob.EV_GRAFT: _abi.TRACE_GRAFT, ob.EV_PRUNE: _abi.TRACE_PRUNE, ob.EV_ADD_PEER: _abi.TRACE_ADD_PEER,
                   ob.EV_REMOVE_PEER: _abi.TRACE_REMOVE_PEER, ob.EV_JOIN: _abi.TRACE_JOIN,
                   ob.EV_LEAVE: _abi.TRACE_LEAVE}[kind]
            out.append((int(e["x"]), 0, a, b, topic, typ, 0))
    arr = np.zeros(len(out), dtype=Engine.TRACE_DTYPE)
    for q, (ts, mid, a, b, topic, typ, rs) in enumerate(out):
        arr[q] = (ts, mid, a, b, topic, typ, rs, 0)
    return arr[np.lexsort((arr["msg_id"], arr["topic"], arr["reason"], arr["other"], arr["type"], arr["peer"],
                           arr["timestamp"]))]


def run_parity(net, params, th, gp, st, ticks, sched, ring=256, behaviour=None, churn=None, after_tick=None,
               eng=None, after_heartbeat=None, px_log=None, trace=None, trace_log=None, topic_slots=0, gater=None,
               gater_log=None, subs=None, local_only=False, trace_every_round=False,
               max_frontier=0, step=False):
    """Run `ticks` on a fresh engine loaded with `st`'s state and on the
    oracle; assert identical state, seen-set and totals after every tick.
    churn: {tick: [(pairs, up), ...]} applied just before the tick.
    eng: an engine whose state `st` already mirrors (nothing is pushed).
    after_heartbeat(kk, eng, st, msgs): called once both heartbeats ran.
    With peer exchange on (gp.PeerExchange) the connector runs after every
    tick on both sides and the connections made must agree (appended to
    px_log when given).  trace=(lo, hi): the engine traces routers [lo, hi)
    and its events must equal the oracle's event log per tick (the event
    counts appended to trace_log).  topic_slots > 0: per-topic sub-rings of
    that many slots (ring = T * topic_slots) with member-compacted seen-set
    cells (gsim_msg_config.topic_slots), on both sides.  gater: a
    gsim.PeerGaterParams turned on at both sides (WithPeerGater); its state
    and the copies it dropped must agree after every tick (the per-tick drop
    counts appended to gater_log).  subs: {tick: [(pairs, join), ...]} Join /
    Leave of (peer, topic) pairs applied just before the tick, after churn.
    local_only: `eng` holds only some shards of the network (one shard per
    process): the parts they own are compared, the totals in full.
    step: the engine runs each tick with one gsim_step call (refresh,
    heartbeat and the rounds with their publications) instead of the
    per-phase calls.  max_frontier: gsim_msg_config.max_frontier (the claim / forwarder list
    bound of member-compacted layouts: small values force their overflow
    fallbacks).  trace_every_round: the engine's trace is read after every round (events
    stamped after the last round run stay for a later read, resolved once)
    and the tick's reads together must equal the oracle's log."""
    from gsim.engine import Engine
    pushed = eng is None
    if eng is None:
        eng = Engine(params, th, gossip=gp)
    try:
        if pushed:
            eng.load_graph(net)
            eng.set_seed(SEED)
            st.push_to_engine(eng)
        if topic_slots:
            ring = st.T * topic_slots
        eng.msgs_init(ring, R, T0, Second, topic_slots=topic_slots, max_frontier=max_frontier)
        msgs = ob.Msgs(net.n, st.T, ring, R, T0, Second, behaviour=behaviour, topic_slots=topic_slots)
        if trace is not None:
            eng.trace_config(trace[0], trace[1], 1 << 22)
            msgs.log()
        if behaviour is not None:
            eng.set_peer_behaviour(behaviour)
        if gater is not None:
            eng.set_peer_gater(gater)
            st.enable_gater(gater)
        lib = ob.load()
        for kk in ticks:
            now = tick_time(kk)
            parts = []
            for (pairs, up) in (churn or {}).get(kk, []):
                st.churn(pairs, up=up, now=now - Second // 2)
                eng.set_connections(pairs, up=up, now=now - Second // 2)
            for (pairs, join) in (subs or {}).get(kk, []):
                st.set_subscriptions(pairs, join, kk, now - Second // 2, SEED)
                eng.set_subscriptions(pairs, join, kk, now - Second // 2)
            if step:
                eng.step(kk, 1, {g: sched[g] for g in range(kk * R, kk * R + R) if g in sched})
            else:
                eng.refresh_scores(now)
                eng.heartbeat(kk, now)
            v = st.view()
            lib.orc_refresh_scores(v, now)
            if gater is not None:
                st.gater_decay(now)
            msgs.penalties(st, now)
            lib.orc_ip_colocation(v)
            lib.orc_compute_scores(v)
            msgs.heartbeat(st, kk, now, SEED)
            if after_heartbeat:
                after_heartbeat(kk, eng, st, msgs)
            for g in range(kk * R, kk * R + R):
                for msg in sched.get(g, []):
                    mid, t, o, inv = msg[:4]
                    msgs.publish(st, mid, t, o, inv, g, vdelay=msg[4] if len(msg) > 4 else 0)
                if g in sched and not step:
                    eng.publish(sched[g], g)
                msgs.round(st, g)
                if not step:
                    eng.round(g)
                if trace is not None and trace_every_round:
                    parts.append(eng.trace_read())
            assert eng.msg_stats() == msgs.stats, f"totals differ at tick {kk}: {eng.msg_stats()} vs {msgs.stats}"
            seen = eng.read(_abi.F_SEEN, into=msgs.seen.copy()) if local_only else eng.read(_abi.F_SEEN)
            lput = eng.read(_abi.F_LASTPUT, into=msgs.lastput.copy()) if local_only else eng.read(_abi.F_LASTPUT)
            assert np.array_equal(seen, msgs.seen), f"seen-set differs at tick {kk}"
            assert np.array_equal(lput, msgs.lastput), f"mcache puts differ at tick {kk}"
            gpu = ob.NetState(net, params, thresholds=th, gossip=gp)
            gpu.pull_from_engine(eng, base=st if local_only else None)
            assert_same(st, gpu)
            if trace is not None:
                got, want = eng.trace_read(), oracle_trace(msgs.events(), msgs, trace[0], trace[1])
                if parts:
                    got = np.concatenate(parts + [got])
                    got = got[np.lexsort((got["msg_id"], got["topic"], got["reason"], got["other"], got["type"],
                                          got["peer"], got["timestamp"]))]
                assert len(got) == len(want), f"trace length differs at tick {kk}: {len(got)} vs {len(want)}"
                for f in ("timestamp", "msg_id", "peer", "other", "topic", "type", "reason"):
                    bad = np.nonzero(got[f] != want[f])[0]
                    assert len(bad) == 0, (f"trace field {f} differs at tick {kk}: first at {bad[:1]}: "
                                           f"{got[max(0, bad[0] - 2):bad[0] + 3]} vs {want[max(0, bad[0] - 2):bad[0] + 3]}")
                if trace_log is not None:
                    rpc = (want["type"] == _abi.TRACE_SEND_RPC) | (want["type"] == _abi.TRACE_RECV_RPC)
                    trace_log.append((np.bincount(want["type"], minlength=13),
                                      np.bincount(want["reason"][rpc], minlength=3)))
            if gater is not None:
                got, want = eng.gater_read(), st.gater_read()
                for f in want:
                    a_, b_ = got[f], want[f]
                    if a_.dtype.itemsize == 8:
                        a_, b_ = a_.view(np.uint64), b_.view(np.uint64)
                    bad = np.argwhere(a_ != b_)
                    assert len(bad) == 0, f"gater {f} differs at tick {kk}: first at {bad[:1].tolist()}"
                assert eng.gater_throttled() == st.gater_throttled(), f"gater drops differ at tick {kk}"
                if gater_log is not None:
                    gater_log.append(st.gater_throttled())
            if gp.PeerExchange:
                t_px = now + Second // 2
                got, want = eng.px_connect(t_px), st.px_connect(t_px)
                assert np.array_equal(got, want), f"PX connections differ after tick {kk}: {len(got)} vs {len(want)}"
                if px_log is not None:
                    px_log.append(len(want))
            if after_tick:
                after_tick(kk, st, msgs)
        return msgs, eng.gossip_stats()
    finally:
        eng.close()


def subscribed_schedule(rng, ticks, net, T, rate, inv_frac, member_only=True, verdicts=None, vdelays=None):
    """Poisson(rate) publications per topic per tick at uniform rounds; the
    origin is a uniform member of the topic (or any peer).  The verdict is
    reject with probability inv_frac, or drawn from `verdicts` (probabilities
    of accept / reject / ignore / throttle / signature) when given.  vdelays:
    validation latencies (rounds) drawn uniformly per message, as a fifth
    tuple element (gsim_msg.vdelay)."""
    sched, mid = {}, 0
    members = [np.nonzero((net.sub >> np.uint64(t)) & np.uint64(1))[0] for t in range(T)]
    for k in ticks:
        for r in range(R):
            g = k * R + r
            batch = []
            for t in range(T):
                pool = members[t] if member_only and len(members[t]) else np.arange(net.n)
                for _ in range(rng.poisson(rate / R)):
                    o = int(pool[rng.integers(0, len(pool))])
                    v = (int(rng.choice(len(verdicts), p=verdicts)) if verdicts is not None
                         else int(rng.random() < inv_frac))
                    if vdelays is not None:
                        batch.append((mid, t, o, v, int(vdelays[rng.integers(0, len(vdelays))])))
                    else:
                        batch.append((mid, t, o, v))
                    mid += 1
            if batch:
                sched[g] = batch
    return sched
