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


def run_parity(net, params, th, gp, st, ticks, sched, ring=256, behaviour=None, churn=None, after_tick=None,
               eng=None, after_heartbeat=None, px_log=None):
    """Run `ticks` on a fresh engine loaded with `st`'s state and on the
    oracle; assert identical state, seen-set and totals after every tick.
    churn: {tick: [(pairs, up), ...]} applied just before the tick.
    eng: an engine whose state `st` already mirrors (nothing is pushed).
    after_heartbeat(kk, eng, st, msgs): called once both heartbeats ran.
    With peer exchange on (gp.PeerExchange) the connector runs after every
    tick on both sides and the connections made must agree (appended to
    px_log when given)."""
    from gsim.engine import Engine
    pushed = eng is None
    if eng is None:
        eng = Engine(params, th, gossip=gp)
    try:
        if pushed:
            eng.load_graph(net)
            eng.set_seed(SEED)
            st.push_to_engine(eng)
        eng.msgs_init(ring, R, T0, Second)
        msgs = ob.Msgs(net.n, st.T, ring, R, T0, Second, behaviour=behaviour)
        if behaviour is not None:
            eng.set_peer_behaviour(behaviour)
        lib = ob.load()
        for kk in ticks:
            now = tick_time(kk)
            for (pairs, up) in (churn or {}).get(kk, []):
                st.churn(pairs, up=up, now=now - Second // 2)
                eng.set_connections(pairs, up=up, now=now - Second // 2)
            eng.refresh_scores(now)
            eng.heartbeat(kk, now)
            v = st.view()
            lib.orc_refresh_scores(v, now)
            msgs.penalties(st, now)
            lib.orc_ip_colocation(v)
            lib.orc_compute_scores(v)
            msgs.heartbeat(st, kk, now, SEED)
            if after_heartbeat:
                after_heartbeat(kk, eng, st, msgs)
            for g in range(kk * R, kk * R + R):
                for (mid, t, o, inv) in sched.get(g, []):
                    msgs.publish(st, mid, t, o, inv, g)
                if g in sched:
                    eng.publish(sched[g], g)
                msgs.round(st, g)
                eng.round(g)
            assert eng.msg_stats() == msgs.stats, f"totals differ at tick {kk}"
            assert np.array_equal(eng.read(_abi.F_SEEN), msgs.seen), f"seen-set differs at tick {kk}"
            assert np.array_equal(eng.read(_abi.F_LASTPUT), msgs.lastput), f"mcache puts differ at tick {kk}"
            gpu = ob.NetState(net, params, thresholds=th, gossip=gp)
            gpu.pull_from_engine(eng)
            assert_same(st, gpu)
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


def subscribed_schedule(rng, ticks, net, T, rate, inv_frac, member_only=True, verdicts=None):
    """Poisson(rate) publications per topic per tick at uniform rounds; the
    origin is a uniform member of the topic (or any peer).  The verdict is
    reject with probability inv_frac, or drawn from `verdicts` (probabilities
    of accept / reject / ignore / throttle / signature) when given."""
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
                    batch.append((mid, t, o, v))
                    mid += 1
            if batch:
                sched[g] = batch
    return sched
