"""gsim_step: whole heartbeat ticks in one call (the
heartbeat timer loop, gossipsub.go:1320-1343).  The engine stepped tick by
tick with one call per tick is bit-exact against the oracle; a multi-tick
call equals the per-phase calls it stands for."""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second
from test_heartbeat import SEED, tick_time

R = 10
T0 = tick_time(0)


@pytest.mark.gpu
@pytest.mark.parametrize("topic_slots", [0, 24])
def test_step_bit_exact(require_gpu, topic_slots):
    """One gsim_step per tick (refresh, heartbeat, ten rounds with their
    publications, every verdict, churn between ticks) against the oracle,
    dense and with member-compacted sub-rings."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from tickrun import restrict_to_subscriptions, run_parity, subscribed_schedule
    rng = np.random.default_rng(606)
    n, T = 3000, 6
    net = graphs.power_law(n, 16, 2.5, 256, seed=61, n_topics=T, i0=1)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 3, seed=62))
    params = beacon_params(T, RetainScore=3 * Second)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300,
                             OpportunisticGraftThreshold=5)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second, OpportunisticGraftTicks=2)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.3)
    restrict_to_subscriptions(st, net)
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 2.0, 0.0, member_only=False,
                                verdicts=[0.8, 0.05, 0.05, 0.05, 0.05])
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 60, replace=False)]
    churn = {2: [(down, False)], 4: [(down, True)]}
    run_parity(net, params, th, gp, st, ticks, sched, ring=T * 24 if topic_slots else 512, churn=churn,
               topic_slots=topic_slots, step=True)


@pytest.mark.gpu
def test_step_many_ticks_equals_phase_calls(require_gpu):
    """gsim_step over three ticks in one call (one upload of the schedule,
    one error read) leaves exactly the state of the per-phase calls:
    delivery totals, seen-set, mcache puts and every score / router field."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import Engine, random_regular
    from tickrun import subscribed_schedule
    rng = np.random.default_rng(707)
    n, k, T = 4000, 32, 4
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-200, PublishThreshold=-400, GraylistThreshold=-800)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    net = random_regular(n, k, seed=70, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.4)
    ticks = list(range(1, 4))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.0, verdicts=(0.8, 0.05, 0.05, 0.05, 0.05))
    engs = []
    for _ in range(2):
        e = Engine(params, th, gossip=gp)
        e.load_graph(net)
        e.set_seed(SEED)
        st.push_to_engine(e)
        e.msgs_init(512, R, T0, Second)
        engs.append(e)
    a, b = engs
    try:
        a.step(1, 3, sched)
        for kk in ticks:
            now = tick_time(kk)
            b.refresh_scores(now)
            b.heartbeat(kk, now)
            for g in range(kk * R, kk * R + R):
                if g in sched:
                    b.publish(sched[g], g)
                b.round(g)
        assert a.msg_stats() == b.msg_stats() and a.msg_stats()[0] > 0
        assert a.gossip_stats() == b.gossip_stats()
        for f in (_abi.F_SEEN, _abi.F_LASTPUT):
            assert np.array_equal(a.read(f), b.read(f))
        sa = ob.NetState(net, params, thresholds=th, gossip=gp)
        sb = ob.NetState(net, params, thresholds=th, gossip=gp)
        sa.pull_from_engine(a)
        sb.pull_from_engine(b)
        for f in sa.TOPIC_FIELDS + sa.EDGE_FIELDS + ("ctl",):
            x, y = getattr(sa, f), getattr(sb, f)
            if x.dtype.itemsize == 8:
                x, y = x.view(np.uint64), y.view(np.uint64)
            assert np.array_equal(x, y), f"state {f} differs"
    finally:
        for e in engs:
            e.close()
