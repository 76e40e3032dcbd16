"""Peer exchange (WithPeerExchange, gossipsub.go:340-350): PRUNEs carry PX
(makePrune 1866-1906), the pruned peer accepts it from peers it scores at
least acceptPXThreshold and queues connection attempts (handlePrune 860-869,
pxConnect 893-939), the connector connects them between ticks (941-973).

CPU part: the oracle's restatement against the reference's rules (which
PRUNEs carry PX, what a PX list may hold, the acceptance threshold, the
connector).  GPU part: the engine against the oracle, bit-exact on every
state array, with the connections made compared after every tick."""
import numpy as np
import pytest

import oracle_binding as ob
from fixtures import beacon_params, synthetic_state
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second

from test_heartbeat import SEED, tick_time


def _px_network(n=600, k=24, T=2, p_mesh=0.7, down_frac=0.25, seed=7, accept=0.0):
    """A random-regular network whose meshes overflow Dhi (Dhi prunes with
    PX) and a quarter of whose connections are down (addresses PX can
    reconnect), every peer in every topic."""
    from gsim.engine import random_regular
    rng = np.random.default_rng(seed)
    net = random_regular(n, k, seed=seed + 1, n_topics=T)
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300,
                             AcceptPXThreshold=accept)
    gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2, PeerExchange=True)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), p_mesh)
    st.bp[rng.random(net.e) < 0.05] = 30.0                 # some negative scores: PRUNEs without PX
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.random(len(und)) < down_frac]
    return net, params, th, gp, st, down


def test_heartbeat_prunes_carry_px_except_negative_score():
    """sendGraftPrune: makePrune(p, topic, doPX && !noPX[p]) — the Dhi
    prunes carry PX, the negative-score prunes (noPX) do not
    (gossipsub.go:1404-1410, 1690)."""
    net, params, th, gp, st, down = _px_network()
    st.churn(down, up=False, now=tick_time(1) - Second // 2)
    lib = ob.load()
    v = st.view()
    now = tick_time(1)
    lib.orc_refresh_scores(v, now)
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    lib.orc_heartbeat(v, 1, now, SEED)
    ctl = st.ctl[0]
    prunes = (ctl & _abi.CTL_PRUNE) != 0
    px = (ctl & _abi.CTL_PX) != 0
    assert px.any() and (prunes & ~px).any()
    assert not (px & ~prunes).any()
    # a PRUNE without PX went to a peer its pruner scores below 0 (the record
    # of the pruner about the receiver sits at the receiver's edge reversed)
    rev = st.rev
    t_idx, e_recv = np.nonzero(prunes & ~px)
    assert (st.score[rev[e_recv]] < 0).all()
    t_idx, e_recv = np.nonzero(px)
    assert (st.score[rev[e_recv]] >= 0).all()


def test_px_attempts_follow_makeprune_and_accept_threshold():
    """Every attempt is to a peer the pruner could list: a topic peer of the
    pruner with score >= 0 other than the pruned peer, at most PrunePeers per
    PRUNE; a pruned peer that scores its pruner below acceptPXThreshold makes
    none (gossipsub.go:862-867)."""
    for accept, expect_any in ((0.0, True), (1e12, False)):
        net, params, th, gp, st, down = _px_network(accept=accept)
        st.churn(down, up=False, now=tick_time(1) - Second // 2)
        lib = ob.load()
        v = st.view()
        now = tick_time(1)
        lib.orc_refresh_scores(v, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
        lib.orc_heartbeat(v, 1, now, SEED)
        marks = st.px.copy()
        assert marks.any() == expect_any
        if not expect_any:
            continue
        owner = net.owner()
        conn = (st.estate & _abi.ES_CONNECTED) != 0
        pruners = {}
        t_idx, e_recv = np.nonzero((st.ctl[0] & _abi.CTL_PX) != 0)
        for t, er in zip(t_idx, e_recv):
            pruners.setdefault(int(owner[er]), set()).add(int(net.col[er]))   # receiver -> its PX pruners
        for e in np.nonzero(marks)[0]:
            p, x = int(owner[e]), int(net.col[e])
            assert not conn[e], "pxConnect skips peers already connected"
            # x is a neighbour of one of p's PX pruners
            ok = False
            for j in pruners.get(p, ()):
                row = net.col[net.row_ptr[j]:net.row_ptr[j + 1]]
                ok |= x in row and x != p
            assert ok
        # connector: every marked pair connects once, the asking side dials
        before = st.estate.copy()
        made = st.px_connect(now + Second // 2)
        assert len(made) > 0
        for d, q in made:
            e = int(np.searchsorted(net.col[net.row_ptr[d]:net.row_ptr[d + 1]], q)) + int(net.row_ptr[d])
            assert net.col[e] == q and not (before[e] & _abi.ES_CONNECTED)
            assert st.estate[e] & _abi.ES_CONNECTED and st.estate[st.rev[e]] & _abi.ES_CONNECTED
            assert net.outbound[e] == 1 and net.outbound[st.rev[e]] == 0
        assert not st.px.any()


@pytest.mark.gpu
@pytest.mark.parametrize("T,accept", [(2, 0.0), (5, 2.0)])
def test_px_bit_exact(require_gpu, T, accept):
    """Ticks with propagation and gossip, PX on: the heartbeat's Dhi prunes
    and handleGraft's mesh-full replies carry PX, the connector reconnects
    known addresses between ticks; state, seen-set and the connections made
    bit-exact against the oracle per tick."""
    from tickrun import run_parity, subscribed_schedule
    net, params, th, gp, st, down = _px_network(n=800, k=24, T=T, accept=accept, seed=11 + T)
    rng = np.random.default_rng(5 + T)
    ticks = list(range(1, 7))
    sched = subscribed_schedule(rng, ticks, net, T, 3.0, 0.02)
    churn = {1: [(down, False)]}
    log = []
    run_parity(net, params, th, gp, st, ticks, sched, ring=512, churn=churn, px_log=log)
    assert sum(log) > 0, "PX made connections"


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [2, 3])
def test_px_sharded_bit_exact(require_gpu, shards):
    """Peer exchange on a graph-sharded network: PRUNEs with PX to a peer of
    another shard carry their lists there (handlePrune's acceptPXThreshold and
    pxConnect's known-address check run at the pruned peer's shard), and the
    connector resolves every shard's attempts once (gsim_group_px_connect):
    state, seen-set and the connections made bit-exact against the oracle."""
    from gsim.shard import ShardedEngine
    from tickrun import SEED, run_parity, subscribed_schedule
    net, params, th, gp, st, down = _px_network(n=900, k=24, T=3, accept=1.0, seed=41 + shards)
    rng = np.random.default_rng(50 + shards)
    eng = ShardedEngine(params, th, gossip=gp, shards=shards)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, 3, 3.0, 0.02)
    churn = {1: [(down, False)]}
    log = []
    run_parity(net, params, th, gp, st, ticks, sched, ring=512, churn=churn, px_log=log, eng=eng)
    assert sum(log) > 0, "PX made connections"
