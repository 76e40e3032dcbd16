"""Dynamic subscriptions: Join / Leave (gossipsub.go:1047-1124) with the
subscription announcements other routers see (pubsub.go:1051-1079)
(SURVEY.md §8(f) row 4).

CPU part: the oracle's Join / Leave against the reference's rules — the
fanout becomes the mesh (negative scores and backoffs dropped, topped up to D
with getPeers), tracer.Graft + GRAFT to each, fanout and lastpub deleted; a
Join without a fanout takes getPeers(D); Leave prunes every mesh peer with an
UnsubscribeBackoff at both ends; a router drops messages of a topic it left.

GPU part: the engine bit-exact against the oracle over ticks with Joins and
Leaves mixed with fanout publishers, gossip and the trace (JOIN / LEAVE /
GRAFT / PRUNE events), on a dense layout and on sub-rings with topic slots
(a Join may grow a peer's slot mask)."""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second
from test_delivery import R, T0, delivery_params
from test_fanout import fanout_net, row, tick, unsubscribe
from test_heartbeat import SEED, tick_time


def test_join_turns_the_fanout_into_the_mesh():
    net, st = fanout_net(ttl=60 * Second)
    msgs = ob.Msgs(net.n, 2, 64, R, T0, Second)
    for kk in range(1, 3):
        tick(st, msgs, kk)
    o = 7                                             # not joined to topic 1: publishes to a fanout
    b, en = row(net, o)
    tick(st, msgs, 3, sched={3 * R: [(1, 1, o, 0)]})
    fan = b + np.nonzero(st.tflags[1, b:en] & _abi.TF_FANOUT)[0]
    assert len(fan) == 6 and st.fan_topics[o] == 2
    st.invalid[1, fan[0]] = 3.0                       # dropped: negative (live) score, P4
    assert ob.load().orc_score_edge(st.view(), int(fan[0])) < 0
    st.backoff[1, fan[1]] = tick_time(4)              # dropped: a backoff entry
    now = tick_time(4) - Second // 2
    st.set_subscriptions([(o, 1)], True, 4, now, SEED)
    assert (net.sub[o] >> np.uint64(1)) & np.uint64(1)
    mesh = b + np.nonzero(st.tflags[1, b:en] & _abi.TF_MESH)[0]
    assert not (st.tflags[1, b:en] & _abi.TF_FANOUT).any()
    assert st.fan_topics[o] == 0 and st.lastpub[o, 1] == 0
    assert set(fan[2:]) <= set(mesh), "the remaining fanout peers are kept"
    assert fan[0] not in mesh and fan[1] not in mesh
    assert len(mesh) == 6, "topped up to D"
    for e in mesh:
        assert st.ctl[0, 1, st.rev[e]] & _abi.CTL_GRAFT, "a GRAFT to every mesh peer"
        assert st.tflags[1, e] & _abi.TF_IN_MESH, "tracer.Graft"
    st.set_subscriptions([(o, 1)], True, 4, now, SEED)        # already joined: no-op
    assert (b + np.nonzero(st.tflags[1, b:en] & _abi.TF_MESH)[0] == mesh).all()


def test_join_filters_on_the_live_score():
    """Join's fanout filter and getPeers call the live gs.score.Score(p)
    (gossipsub.go:1063, 1076, 1091), not the snapshot of the last refresh: a
    candidate whose invalid deliveries since that refresh made its score
    negative is not grafted, although its snapshot score is still >= 0."""
    lib = ob.load()
    net, st = fanout_net()
    msgs = ob.Msgs(net.n, 2, 64, R, T0, Second)
    for kk in range(1, 3):
        tick(st, msgs, kk)
    o = 3
    b, en = row(net, o)
    cands = [e for e in range(b, en) if (net.sub[net.col[e]] >> np.uint64(1)) & np.uint64(1)]
    assert len(cands) > 6
    bad = cands[:len(cands) - 6]                  # leave exactly D good candidates
    v = st.view()
    for e in bad:
        st.invalid[1, e] = 3.0                    # RejectMessage deliveries since the refresh (P4)
        assert st.score[e] >= 0 and lib.orc_score_edge(v, e) < 0
    st.set_subscriptions([(o, 1)], True, 3, tick_time(3) - Second // 2, SEED)
    mesh = set(b + np.nonzero(st.tflags[1, b:en] & _abi.TF_MESH)[0])
    assert not (mesh & set(bad)), "a negative live score is filtered out"
    assert mesh == set(cands) - set(bad)


def test_join_without_fanout_takes_d_peers():
    net, st = fanout_net()
    o = 3
    b, en = row(net, o)
    st.set_subscriptions([(o, 1)], True, 1, tick_time(1), SEED)
    mesh = np.nonzero(st.tflags[1, b:en] & _abi.TF_MESH)[0]
    assert len(mesh) == 6
    assert all((net.sub[net.col[b + q]] >> np.uint64(1)) & np.uint64(1) for q in mesh), "topic peers only"


def test_leave_prunes_with_the_unsubscribe_backoff():
    net, st = fanout_net()
    gp = GossipSubParams(D=6, Dlo=5, Dhi=12)
    msgs = ob.Msgs(net.n, 2, 64, R, T0, Second)
    for kk in range(1, 3):
        tick(st, msgs, kk)
    o = 150
    b, en = row(net, o)
    mesh = b + np.nonzero(st.tflags[0, b:en] & _abi.TF_MESH)[0]
    assert len(mesh) >= gp.Dlo
    now = tick_time(3) - Second // 2
    st.set_subscriptions([(o, 0)], False, 3, now, SEED)
    assert not (net.sub[o] & np.uint64(1))
    assert not (st.tflags[0, b:en] & _abi.TF_MESH).any()
    for e in mesh:
        c = st.ctl[0, 0, st.rev[e]]
        assert (c & _abi.CTL_PRUNE) and (c & _abi.CTL_UNSUB)
        assert st.backoff[0, e] == now + gp.UnsubscribeBackoff
        assert not (st.tflags[0, e] & _abi.TF_IN_MESH), "tracer.Prune"
    # the pruned peers obey the PRUNE's backoff (UnsubscribeBackoff / 1s)
    ob.load().orc_handle_control(st.view(), 0, now)
    for e in mesh:
        re = st.rev[e]
        assert not (st.tflags[0, re] & _abi.TF_MESH)
        assert st.backoff[0, re] == now + gp.UnsubscribeBackoff


def test_leave_prunes_carry_peer_exchange():
    """With WithPeerExchange, Leave's sendPrune(p, topic, true) builds its
    PRUNE with makePrune(p, topic, gs.doPX, true) (gossipsub.go:1118,
    1132-1133): a PX list of up to PrunePeers topic peers other than p with a
    live score >= 0 (1866-1906).  The pruned peers take it up with the tick's
    control: at the connector, each one that scores the leaver >=
    acceptPXThreshold asks for every listed peer it knows and is not
    connected to."""
    from gsim.engine import random_regular
    net = random_regular(300, 12, seed=11, n_topics=2)
    gp = GossipSubParams(D=6, Dlo=5, Dhi=12, PeerExchange=True, PrunePeers=4)
    from test_fanout import TH
    st = ob.NetState(net, delivery_params(2), thresholds=TH, gossip=gp)
    msgs = ob.Msgs(net.n, 2, 64, R, T0, Second)
    for kk in range(1, 3):
        tick(st, msgs, kk)
    o = 150
    b, en = row(net, o)
    mesh = b + np.nonzero(st.tflags[0, b:en] & _abi.TF_MESH)[0]
    assert len(mesh) >= gp.Dlo
    msgs.log()
    now = tick_time(3) - Second // 2
    st.set_subscriptions([(o, 0)], False, 3, now, SEED)
    ev = msgs.events()
    px = ev[ev["kind"] == ob.EV_PX_PEER]
    lib = ob.load()
    for e in mesh:
        c = st.ctl[0, 0, st.rev[e]]
        assert (c & _abi.CTL_PRUNE) and (c & _abi.CTL_UNSUB) and (c & _abi.CTL_PX)
        lst = px[px["mid"] == net.col[e]]
        assert len(lst) == gp.PrunePeers and list(lst["g"]) == list(range(gp.PrunePeers))
        assert all(lst["a"] == o) and all(lst["topic"] == 0)
        assert net.col[e] not in lst["b"], "xp != p"
        for y in lst["b"]:
            ey = b + int(np.searchsorted(net.col[b:en], y))
            assert net.col[ey] == y and (net.sub[y] & np.uint64(1))
            assert lib.orc_score_edge(st.view(), ey) >= 0
    # the connector: a listed peer whose address the pruned peer knows is one it
    # is connected to here (no churn): no connection attempt comes of the lists
    assert len(st.px_connect(tick_time(3) + Second // 2)) == 0


def test_a_router_drops_messages_of_a_topic_it_left():
    net, st = fanout_net()
    msgs = ob.Msgs(net.n, 2, 64, R, T0, Second)
    for kk in range(1, 3):
        tick(st, msgs, kk)
    o = 200
    st.set_subscriptions([(o, 0)], False, 3, tick_time(3) - Second // 2, SEED)
    tick(st, msgs, 3, sched={3 * R + 1: [(5, 0, 201, 0)]})
    assert msgs.seen[5, o] == ob.UNSEEN, "the copies to the peer that left were skipped"
    subscribed = (net.sub & np.uint64(1)).astype(bool)
    assert (msgs.seen[5, subscribed] != ob.UNSEEN).all()


# ---- GPU parity -------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("topic_slots,shards,px", [(0, 0, False), (80, 0, False), (0, 3, False), (0, 0, True),
                                                   (0, 3, True)])
def test_join_leave_bit_exact(require_gpu, topic_slots, shards, px):
    """Joins (with and without a fanout) and Leaves between ticks, fanout
    publishers, gossip, churn and the trace: every state array, the seen-set,
    the totals and the JOIN / LEAVE / GRAFT / PRUNE events bit-exact — on one
    engine and on 3 shards (GRAFT / PRUNE to other shards' peers leave with
    the heartbeat's control exchange)."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import restrict_to_subscriptions, run_parity, subscribed_schedule
    n, k, T = 900, 16, 3
    rng = np.random.default_rng(515 + topic_slots)
    params = beacon_params(T)
    gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2, FanoutTTL=30 * Second, PeerExchange=px)
    th = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-100, GraylistThreshold=-400)
    net = random_regular(n, k, seed=91, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 6 / k)
    for t in range(1, T):
        unsubscribe(net, st, np.nonzero(rng.random(n) < 0.3)[0], t)
    restrict_to_subscriptions(st, net)
    ticks = list(range(1, 8))
    # publishers are any peers: non-members build fanouts that later Joins turn into meshes
    sched = subscribed_schedule(rng, ticks, net, T, 6.0, 0.05, member_only=False)

    def members(t, want):
        return np.nonzero(((net.sub >> np.uint64(t)) & np.uint64(1)).astype(bool) == want)[0]

    subs = {}
    for kk, join in ((3, True), (4, False), (5, True), (6, False)):
        ev = []
        for t in range(T):
            pool = members(t, not join)
            for p in rng.choice(pool, size=min(12, len(pool)), replace=False):
                ev.append((int(p), t))
        subs[kk] = [(np.array(ev, dtype=np.uint32), join)]
    log = []
    eng = None
    if shards:
        from gsim.shard import ShardedEngine
        from tickrun import SEED as TSEED
        eng = ShardedEngine(params, th, gossip=gp, shards=shards)
        eng.load_graph(net)
        eng.set_seed(TSEED)
        st.push_to_engine(eng)
    run_parity(net, params, th, gp, st, ticks, sched, ring=256, subs=subs, trace=(0, n),
               trace_log=log, topic_slots=topic_slots, eng=eng)
    total = np.sum([x[0] for x in log], axis=0)
    assert total[_abi.TRACE_JOIN] > 0 and total[_abi.TRACE_LEAVE] > 0
