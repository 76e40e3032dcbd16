"""Connection churn between ticks: the router's and the score tracer's
RemovePeer / AddPeer on both endpoints (gossipsub.go:525-567,
score.go:595-644; driven by handleDeadPeers pubsub.go:711-759).

CPU part: the oracle's network-level churn against the reference's
RemovePeer rules, as score_test.go TestScoreRetention (score_test.go:897-941)
asserts them for one peer: a positive score is dropped, a non-positive one
is retained for RetainScore with P2 reset and the P3b penalty, and purged
by refreshScores after it expires.  GPU part: gsim_set_connections against
the oracle, bit-exact, through ticks with propagation and gossip.
"""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second
from test_delivery import R, T0, delivery_params
from test_heartbeat import SEED, tick_time

RETAIN = 3 * Second


def churn_net(n=200, k=8):
    from gsim.engine import random_regular
    net = random_regular(n, k, seed=5, n_topics=1)
    params = delivery_params(1)
    params.RetainScore = RETAIN
    st = ob.NetState(net, params, thresholds=PeerScoreThresholds(GraylistThreshold=-100),
                     gossip=GossipSubParams(D=6, Dlo=5, Dhi=12))
    st.estate[:] = _abi.ES_TRACKED | _abi.ES_CONNECTED
    return net, st


def edge(net, i, j):
    b, en = int(net.row_ptr[i]), int(net.row_ptr[i + 1])
    return b + int(np.searchsorted(net.col[b:en], j))


def test_remove_drops_positive_retains_non_positive_and_purges():
    net, st = churn_net()
    a = 3
    b = int(net.col[net.row_ptr[a]])
    eab, eba = edge(net, a, b), edge(net, b, a)
    now = tick_time(2)
    # a's record of b: positive (first deliveries); b's record of a: negative,
    # in mesh and active below the delivery threshold (P3b applies)
    st.first[0, eab] = 10.0
    st.tflags[0, eab] = _abi.TF_MESH | _abi.TF_IN_MESH
    st.first[0, eba] = 2.0
    st.invalid[0, eba] = 3.0
    st.meshd[0, eba] = 0.25
    st.fail[0, eba] = 1.0
    st.tflags[0, eba] = _abi.TF_MESH | _abi.TF_IN_MESH | _abi.TF_ACTIVE
    lib = ob.load()
    assert lib.orc_score_edge(st.view(), eab) > 0
    assert lib.orc_score_edge(st.view(), eba) <= 0
    st.ctl[:, 0, eab] = _abi.CTL_GRAFT
    st.churn([(a, b)], up=False, now=now)
    # router: out of the mesh both ways, pending control dropped
    assert not (st.tflags[0, eab] & _abi.TF_MESH) and not (st.tflags[0, eba] & _abi.TF_MESH)
    assert (st.ctl[:, 0, eab] == 0).all()
    # positive score dropped
    assert st.estate[eab] == 0 and st.first[0, eab] == 0.0
    # non-positive retained: P2 reset, P3b (threshold 1 - 0.25)^2 added, inMesh off
    assert st.estate[eba] == _abi.ES_TRACKED
    assert st.expire[eba] == now + RETAIN
    assert st.first[0, eba] == 0.0
    assert st.fail[0, eba] == 1.0 + 0.75 * 0.75
    assert not (st.tflags[0, eba] & _abi.TF_IN_MESH)
    # still retained before the expiry, purged after it
    lib.orc_refresh_scores(st.view(), now + RETAIN)
    assert st.estate[eba] == _abi.ES_TRACKED
    lib.orc_refresh_scores(st.view(), now + RETAIN + Second)
    assert st.estate[eba] == 0
    # reconnect: fresh records on both sides
    st.churn([(b, a)], up=True, now=now + 5 * Second)
    assert st.estate[eab] == st.estate[eba] == _abi.ES_TRACKED | _abi.ES_CONNECTED
    assert st.invalid[0, eba] == 0.0 and st.fail[0, eba] == 0.0


def test_reconnect_reuses_retained_record():
    """AddPeer within RetainScore brings the retained counters back (score.go:595-609)."""
    net, st = churn_net()
    a = 10
    b = int(net.col[net.row_ptr[a] + 1])
    eab = edge(net, a, b)
    st.invalid[0, eab] = 4.0
    st.churn([(a, b)], up=False, now=tick_time(1))
    assert st.estate[eab] == _abi.ES_TRACKED
    st.churn([(a, b)], up=True, now=tick_time(2))
    assert st.estate[eab] == _abi.ES_TRACKED | _abi.ES_CONNECTED
    assert st.invalid[0, eab] == 4.0


def test_disconnected_peer_gets_no_messages():
    """A peer whose every connection went down is outside every mesh and
    receives nothing; after reconnecting, the heartbeat grafts it again."""
    from test_heartbeat import run_tick_oracle
    net, st = churn_net(n=300, k=12)
    for kk in range(1, 4):
        run_tick_oracle(st, kk)
    p = 17
    pairs = [(p, int(j)) for j in net.col[net.row_ptr[p]:net.row_ptr[p + 1]]]
    st.churn(pairs, up=False, now=tick_time(3) + Second // 2)
    msgs = ob.Msgs(net.n, 1, 64, R, T0, Second)
    lib = ob.load()
    k = 4
    v = st.view()
    lib.orc_refresh_scores(v, tick_time(k))
    lib.orc_compute_scores(v)
    msgs.heartbeat(st, k, tick_time(k), SEED)
    b, en = int(net.row_ptr[p]), int(net.row_ptr[p + 1])
    assert not (st.tflags[0, b:en] & _abi.TF_MESH).any(), "nobody grafts a disconnected peer"
    for g in range(k * R, k * R + R):
        if g == k * R:
            msgs.publish(st, 1, 0, 0 if p != 0 else 1, 0, g)
        msgs.round(st, g)
    assert msgs.seen[1, p] == ob.UNSEEN
    assert (msgs.seen[1] != ob.UNSEEN).sum() == net.n - 1
    st.churn(pairs, up=True, now=tick_time(k) + Second // 2)
    lib.orc_refresh_scores(v, tick_time(k + 1))
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    msgs.heartbeat(st, k + 1, tick_time(k + 1), SEED)
    assert (st.tflags[0, b:en] & _abi.TF_MESH).any(), "Dlo graft after reconnecting"


# ---- GPU parity -------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("n,k,T,nticks,rate,churn_frac", [
    (1200, 16, 2, 9, 8, 0.02),
    (2500, 32, 3, 8, 10, 0.05),
])
def test_churn_ticks_bit_exact(require_gpu, n, k, T, nticks, rate, churn_frac):
    """Connections go down and come back between ticks while messages and
    gossip flow: every state array, the seen-set and the totals bit-exact.
    RetainScore = 3 s, so retained records are purged within the run."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import Engine, random_regular
    from test_delivery import _schedule
    from test_heartbeat import assert_same
    rng = np.random.default_rng(n * 3 + k)
    params = beacon_params(T, RetainScore=RETAIN)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-50, GraylistThreshold=-300)
    net = random_regular(n, k, seed=n + 7, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    st.bp[rng.random(net.e) < 0.05] = 12.0          # some non-positive scores: retained on removal
    msgs = ob.Msgs(n, T, 256, R, T0, Second)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    eng.msgs_init(256, R, T0, Second)
    ticks = list(range(1, nticks + 1))
    sched = _schedule(rng, ticks, T, R, rate, 0.05, n)
    lib = ob.load()
    # undirected connections (a < b)
    src = np.repeat(np.arange(n, dtype=np.uint32), np.diff(net.row_ptr).astype(np.int64))
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = []
    n_retained = 0
    for kk in ticks:
        now = tick_time(kk)
        # churn between ticks: some connections go down, earlier ones come back
        t_churn = now - Second // 2
        if kk >= 2:
            if down:
                up = down.pop(0)
                st.churn(up, up=True, now=t_churn)
                eng.set_connections(up, up=True, now=t_churn)
            pick = und[rng.choice(len(und), size=max(1, int(churn_frac * len(und))), replace=False)]
            busy = {tuple(x) for batch in down for x in batch}
            pick = np.array([x for x in pick if tuple(x) not in busy], dtype=np.uint32)
            st.churn(pick, up=False, now=t_churn)
            eng.set_connections(pick, up=False, now=t_churn)
            n_retained += int((((st.estate & _abi.ES_TRACKED) != 0) & ((st.estate & _abi.ES_CONNECTED) == 0)).sum())
            down.append(pick)
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
    assert n_retained > 0, "some removals were retained"
    eng.close()


@pytest.mark.gpu
def test_set_connections_rejects_bad_lists(require_gpu):
    """gsim_set_connections fails, changing nothing, on a pair that is not a
    connection or a connection listed twice (in either order: the checks run
    on the device, the listed connections marked in an edge bitmap that is
    cleared again); a good list afterwards applies as the oracle does."""
    from gsim.engine import Engine
    from test_heartbeat import assert_same
    net, st = churn_net()
    params = delivery_params(1)
    params.RetainScore = RETAIN
    eng = Engine(params, PeerScoreThresholds(GraylistThreshold=-100), gossip=GossipSubParams(D=6, Dlo=5, Dhi=12))
    eng.load_graph(net)
    st.push_to_engine(eng)
    a = 3
    b, c = (int(x) for x in net.col[net.row_ptr[a]:net.row_ptr[a] + 2])
    non = next(j for j in range(net.n) if j != a and j not in set(net.col[net.row_ptr[a]:net.row_ptr[a + 1]].tolist()))
    now = tick_time(2)
    for bad, what in (([(a, b), (a, c), (b, a)], "listed twice"), ([(a, c), (a, c)], "listed twice"),
                      ([(a, b), (a, non)], "not a connection"), ([(a, a)], "not a connection")):
        with pytest.raises(ValueError, match=what):
            eng.set_connections(bad, up=False, now=now)
        gpu = ob.NetState(net, params, thresholds=PeerScoreThresholds(GraylistThreshold=-100),
                          gossip=GossipSubParams(D=6, Dlo=5, Dhi=12))
        gpu.pull_from_engine(eng)
        assert_same(st, gpu)
    good = [(a, b), (c, a)]
    eng.set_connections(good, up=False, now=now)
    st.churn(good, up=False, now=now)
    gpu = ob.NetState(net, params, thresholds=PeerScoreThresholds(GraylistThreshold=-100),
                      gossip=GossipSubParams(D=6, Dlo=5, Dhi=12))
    gpu.pull_from_engine(eng)
    assert_same(st, gpu)
    eng.close()
