"""Fanout and flood publishing: Publish from a peer that has not joined the
topic goes to its fanout (gossipsub.go:1011-1028), the heartbeat expires and
maintains fanouts and gossips for them (1558-1596); WithFloodPublish sends an
origin's own message to every topic peer with score >= publishThreshold
(989-995).

CPU part: the oracle's behaviour against those rules.  GPU part: the engine
against the oracle, bit-exact, over ticks with fanout publishers, expiry and
flood publishing.
"""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second
from test_delivery import R, T0, delivery_params
from test_heartbeat import SEED, tick_time

TH = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-60, GraylistThreshold=-100)


def unsubscribe(net, st, peers, t):
    """peers leave topic t before the run (and are in no mesh of it)."""
    for p in peers:
        net.sub[p] &= ~np.uint64(1 << t)
    rev = st.rev
    for p in peers:
        for e in range(int(net.row_ptr[p]), int(net.row_ptr[p + 1])):
            st.tflags[t, e] &= ~np.uint8(_abi.TF_MESH)
            st.tflags[t, rev[e]] &= ~np.uint8(_abi.TF_MESH)


def fanout_net(n=300, k=12, flood=False, ttl=3 * Second):
    from gsim.engine import random_regular
    net = random_regular(n, k, seed=11, n_topics=2)
    gp = GossipSubParams(D=6, Dlo=5, Dhi=12, FanoutTTL=ttl, FloodPublish=flood)
    st = ob.NetState(net, delivery_params(2), thresholds=TH, gossip=gp)
    unsubscribe(net, st, range(0, 40), 1)
    return net, st


def tick(st, msgs, kk, sched=None, before_heartbeat=None):
    lib = ob.load()
    v = st.view()
    now = tick_time(kk)
    lib.orc_refresh_scores(v, now)
    msgs.penalties(st, now)
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    if before_heartbeat:
        before_heartbeat()
    msgs.heartbeat(st, kk, now, SEED)
    for g in range(kk * R, kk * R + R):
        for (mid, t, o, inv) in (sched or {}).get(g, []):
            msgs.publish(st, mid, t, o, inv, g)
        msgs.round(st, g)


def row(net, p):
    return int(net.row_ptr[p]), int(net.row_ptr[p + 1])


def test_publish_without_joining_uses_fanout_then_expires():
    net, st = fanout_net()
    msgs = ob.Msgs(net.n, 2, 64, R, T0, Second)
    for kk in range(1, 4):
        tick(st, msgs, kk)
    o, k = 5, 4                                   # 5 has not joined topic 1
    b, en = row(net, o)
    assert not (st.tflags[1, b:en] & _abi.TF_MESH).any()
    g = k * R + 1
    tick(st, msgs, k, sched={g: [(9, 1, o, 0)]})
    fan = (st.tflags[1, b:en] & _abi.TF_FANOUT) != 0
    assert fan.sum() == 6, "getPeers(topic, D) with score >= publishThreshold"
    assert all((net.sub[net.col[b + q]] >> np.uint64(1)) & np.uint64(1) for q in np.nonzero(fan)[0])
    assert st.fan_topics[o] == 2
    assert st.lastpub[o, 1] == msgs.round_time(g)
    subscribed = ((net.sub >> np.uint64(1)) & np.uint64(1)).astype(bool)
    seen = msgs.seen[9] != ob.UNSEEN
    assert seen[subscribed].all(), "every topic member got the message"
    assert not seen[~subscribed & (np.arange(net.n) != o)].any()
    # the fanout is kept while published to, expired after FanoutTTL (3 s)
    tick(st, msgs, k + 1)
    assert ((st.tflags[1, b:en] & _abi.TF_FANOUT) != 0).sum() == 6
    for kk in range(k + 2, k + 5):
        tick(st, msgs, kk)
    assert st.fan_topics[o] == 0 and st.lastpub[o, 1] == 0
    assert not (st.tflags[1, b:en] & _abi.TF_FANOUT).any()


def test_fanout_drops_low_scores_and_tops_up():
    net, st = fanout_net(ttl=60 * Second)
    msgs = ob.Msgs(net.n, 2, 64, R, T0, Second)
    for kk in range(1, 3):
        tick(st, msgs, kk)
    o = 7
    b, en = row(net, o)
    tick(st, msgs, 3, sched={3 * R: [(1, 1, o, 0)]})
    fan = np.nonzero(st.tflags[1, b:en] & _abi.TF_FANOUT)[0]
    victim = b + int(fan[0])

    def sink():
        st.score[victim] = -1000.0                # below publishThreshold at this heartbeat

    tick(st, msgs, 4, before_heartbeat=sink)
    assert not (st.tflags[1, victim] & _abi.TF_FANOUT)
    assert ((st.tflags[1, b:en] & _abi.TF_FANOUT) != 0).sum() == 6, "topped up to D"


def test_flood_publish_reaches_every_topic_peer_first():
    for flood in (False, True):
        net, st = fanout_net(flood=flood)
        msgs = ob.Msgs(net.n, 2, 64, R, T0, Second)
        for kk in range(1, 4):
            tick(st, msgs, kk)
        o, k = 100, 4
        g = k * R
        tick(st, msgs, k, sched={g: [(3, 0, o, 0)]})
        b, en = row(net, o)
        first_hop = (msgs.seen[3, net.col[b:en]] == g + 1).sum()
        mesh = ((st.tflags[0, b:en] & _abi.TF_MESH) != 0).sum()
        if flood:
            assert first_hop == en - b, "flood: every topic peer above publishThreshold"
        else:
            assert first_hop <= max(mesh, 12) and first_hop < en - b


# ---- GPU parity -------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("n,k,T,nticks,rate,flood", [
    (1200, 16, 3, 9, 8, False),
    (1500, 24, 2, 6, 10, True),
])
def test_fanout_ticks_bit_exact(require_gpu, n, k, T, nticks, rate, flood):
    """Non-member publishers (fanout creation, maintenance, expiry after a
    3 s FanoutTTL, fanout gossip) or flood publishing: every state array incl.
    lastpub / fanout topics, the seen-set and the totals bit-exact."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import Engine, random_regular
    from test_delivery import _schedule
    from test_heartbeat import assert_same
    rng = np.random.default_rng(n + 31 * k)
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second, FloodPublish=flood)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
    net = random_regular(n, k, seed=n + 3, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    st.bp[rng.random(net.e) < 0.03] = 12.0
    for t in range(1, T):
        unsubscribe(net, st, np.nonzero(rng.random(n) < 0.2 * t)[0], t)
    msgs = ob.Msgs(n, T, 256, R, T0, Second)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    eng.msgs_init(256, R, T0, Second)
    ticks = list(range(1, nticks + 1))
    # publications only in the first ticks, so fanouts expire at the end
    sched = _schedule(rng, ticks[:-4], T, R, rate, 0.05, n)
    lib = ob.load()
    for kk in ticks:
        now = tick_time(kk)
        eng.refresh_scores(now)
        eng.heartbeat(kk, now)
        v = st.view()
        lib.orc_refresh_scores(v, now)
        msgs.penalties(st, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
        msgs.heartbeat(st, kk, now, SEED)
        for g in range(kk * R, kk * R + R):
            for (mid, t, o, inv) in sched.get(g, []):
                msgs.publish(st, mid, t, o, inv, g)
            if g in sched:
                eng.publish(sched[g], g)
            msgs.round(st, g)
            eng.round(g)
        assert eng.msg_stats() == msgs.stats, f"tick {kk}"
        assert np.array_equal(eng.read(_abi.F_SEEN), msgs.seen), f"seen-set differs at tick {kk}"
        gpu = ob.NetState(net, params, thresholds=th, gossip=gp)
        gpu.pull_from_engine(eng)
        assert_same(st, gpu)
        if kk == nticks - 4 and not flood:
            assert (st.fan_topics != 0).any(), "some publishers used a fanout"
    if not flood:
        assert (st.fan_topics == 0).all() and (st.lastpub == 0).all(), "every fanout expired"
    eng.close()
