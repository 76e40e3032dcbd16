"""Direct peers (WithDirectPeers, gossipsub.go:352-374): never grafted
(1416-1422, 1506-1512, 1540-1545) nor gossiped to (1728-1737), a GRAFT from
one is answered with PRUNE (768-776), every message of a topic they joined is
sent to them (991-1003) and AcceptFrom accepts them whatever their score
(598-609).

CPU part: the oracle against those rules (the reference's
TestDirectPeerFanout / direct-peer tests assert delivery between direct peers
that are not in each other's mesh).  GPU part: engine vs oracle, bit-exact.
"""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second
from test_delivery import R, T0, delivery_params
from test_heartbeat import SEED, tick_time

TH = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-60, GraylistThreshold=-100)


def direct_net(n=300, k=12):
    from gsim.engine import random_regular
    net = random_regular(n, k, seed=21, n_topics=1)
    st = ob.NetState(net, delivery_params(1), thresholds=TH, gossip=GossipSubParams(D=6, Dlo=5, Dhi=12))
    return net, st


def make_direct(net, st, pairs):
    rev = st.rev
    for (a, b) in pairs:
        lo, hi = int(net.row_ptr[a]), int(net.row_ptr[a + 1])
        e = lo + int(np.searchsorted(net.col[lo:hi], b))
        st.direct[e] = 1
        st.direct[rev[e]] = 1


def tick(st, msgs, kk, sched=None, before=None):
    lib = ob.load()
    v = st.view()
    now = tick_time(kk)
    lib.orc_refresh_scores(v, now)
    msgs.penalties(st, now)
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    if before:
        before()
    msgs.heartbeat(st, kk, now, SEED)
    for g in range(kk * R, kk * R + R):
        for (mid, t, o, inv) in (sched or {}).get(g, []):
            msgs.publish(st, mid, t, o, inv, g)
        msgs.round(st, g)


def test_direct_peers_never_meshed_or_gossiped_but_always_sent_to():
    net, st = direct_net()
    a = 10
    pairs = [(a, int(b)) for b in net.col[net.row_ptr[a]:net.row_ptr[a] + 4]]
    make_direct(net, st, pairs)
    msgs = ob.Msgs(net.n, 1, 64, R, T0, Second)
    for kk in range(1, 5):
        tick(st, msgs, kk, sched={kk * R + 1: [(kk, 0, 50 + kk, 0)]})
    d = np.nonzero(st.direct)[0]
    assert not (st.tflags[0, d] & _abi.TF_MESH).any(), "direct links never join a mesh"
    # a message published by a reaches its direct peers in the next round,
    # mesh or not
    k = 5
    g = k * R + 1
    tick(st, msgs, k, sched={g: [(99, 0, a, 0)]})
    slot = 99 % 64
    for (_, b) in pairs:
        assert msgs.seen[slot, b] == g + 1, "direct peers get every message of a joined topic"


def test_graft_from_direct_peer_is_pruned():
    net, st = direct_net()
    a = 3
    b = int(net.col[net.row_ptr[a]])
    make_direct(net, st, [(a, b)])
    lo = int(net.row_ptr[a])
    e = lo + int(np.searchsorted(net.col[lo:int(net.row_ptr[a + 1])], b))
    # b sent a GRAFT to a (a's inbox at a's edge to b)
    st.ctl[0, 0, e] = _abi.CTL_GRAFT
    lib = ob.load()
    lib.orc_compute_scores(st.view())
    lib.orc_handle_control(st.view(), 0, tick_time(1))
    assert not (st.tflags[0, e] & _abi.TF_MESH)
    assert st.ctl[1, 0, st.rev[e]] & _abi.CTL_PRUNE, "answered with PRUNE"
    assert st.backoff[0, e] == 0 and st.bp[e] == 0, "no backoff, no penalty"


def test_direct_peer_accepted_below_graylist():
    net, st = direct_net()
    a = 7
    b = int(net.col[net.row_ptr[a]])
    make_direct(net, st, [(a, b)])
    msgs = ob.Msgs(net.n, 1, 64, R, T0, Second)
    for kk in range(1, 4):
        tick(st, msgs, kk)
    lo = int(net.row_ptr[b])
    eb = lo + int(np.searchsorted(net.col[lo:int(net.row_ptr[b + 1])], a))   # b's edge to a

    def sink():
        st.score[eb] = -1000.0                    # b would graylist a

    g = 4 * R
    tick(st, msgs, 4, sched={g: [(5, 0, a, 0)]}, before=sink)
    assert msgs.seen[5, b] == g + 1, "AcceptAll for a direct peer"


# ---- GPU parity -------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("n,k,T,nticks,frac,flood", [
    (1500, 16, 2, 6, 0.05, False),
    (2000, 32, 2, 5, 0.03, True),
])
def test_direct_ticks_bit_exact(require_gpu, n, k, T, nticks, frac, flood):
    """Random symmetric direct links (some graylisted, some with GRAFTs in
    flight from the synthetic meshes) through ticks with gossip: engine vs
    oracle bit-exact."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import run_parity, subscribed_schedule
    rng = np.random.default_rng(n + k * 3)
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FloodPublish=flood)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-100)
    net = random_regular(n, k, seed=n + 9, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    st.bp[rng.random(net.e) < 0.03] = 40.0          # some graylisted senders
    und = np.nonzero(net.owner() < net.col)[0]
    pick = und[rng.random(len(und)) < frac]
    st.direct[pick] = 1
    st.direct[st.rev[pick]] = 1
    ticks = list(range(1, nticks + 1))
    sched = subscribed_schedule(rng, ticks, net, T, 8, 0.05)
    run_parity(net, params, th, gp, st, ticks, sched, ring=256)
