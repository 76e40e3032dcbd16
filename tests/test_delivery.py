"""Message propagation rounds: publish -> mesh forwarding -> seen-set ->
P2/P3/P4 delivery counters (pushMsg pubsub.go:1118-1162, Publish
gossipsub.go:975-1045, score.go:693-981).

CPU part: behavioural invariants of the oracle restatement (what the
reference's integration tests assert: every subscriber receives each message
once, duplicates are credited, invalid messages are penalised, graylisted
peers are ignored).  GPU part: the engine against the oracle, bit-exact on the
seen-set, the counters and every state array, across heartbeats.
"""
from collections import deque

import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreParams, PeerScoreThresholds, Second, TopicScoreParams
from test_heartbeat import SEED, run_tick_oracle, tick_time

HB = Second
R = 10                       # propagation rounds per heartbeat
T0 = tick_time(0)


def delivery_params(T=1, window=10 * Second):
    tp = TopicScoreParams(TopicWeight=1, TimeInMeshWeight=0.01, TimeInMeshQuantum=Second, TimeInMeshCap=10,
                          FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=0.5,
                          FirstMessageDeliveriesCap=1000,
                          MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=0.5,
                          MeshMessageDeliveriesThreshold=1, MeshMessageDeliveriesCap=1000,
                          MeshMessageDeliveriesActivation=30 * Second, MeshMessageDeliveriesWindow=window,
                          MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=0.5,
                          InvalidMessageDeliveriesWeight=-1, InvalidMessageDeliveriesDecay=0.5)
    p = PeerScoreParams(AppSpecificScore=lambda q: 0.0, AppSpecificWeight=1, DecayInterval=Second,
                        DecayToZero=0.01)
    for t in range(T):
        p.Topics[f"t{t}"] = tp
    return p


def settled_state(n=600, k=16, T=1, window=10 * Second, ticks=3):
    """A network whose meshes formed over `ticks` heartbeats (GRAFT/PRUNE exchanged)."""
    from gsim.engine import random_regular
    net = random_regular(n, k, seed=1, n_topics=T)
    st = ob.NetState(net, delivery_params(T, window), thresholds=PeerScoreThresholds(GraylistThreshold=-100),
                     gossip=GossipSubParams(D=6, Dlo=5, Dhi=12))
    for kk in range(1, ticks + 1):
        run_tick_oracle(st, kk)
    return net, st


def mesh_bfs(net, st, t, origin):
    """Hop distance over the directed mesh graph (j forwards to i over j's mesh)."""
    m = (st.tflags[t] & _abi.TF_MESH) != 0
    dist = np.full(net.n, -1, dtype=np.int64)
    dist[origin] = 0
    q = deque([origin])
    while q:
        j = q.popleft()
        for e in range(int(net.row_ptr[j]), int(net.row_ptr[j + 1])):
            i = int(net.col[e])
            if m[e] and dist[i] < 0:
                dist[i] = dist[j] + 1
                q.append(i)
    return dist


def run_rounds(st, msgs, g0, g1):
    for g in range(g0, g1):
        msgs.round(st, g)


def test_round_clock_matches_control_rounds():
    msgs = ob.Msgs(10, 1, 4, R, T0, HB)
    assert msgs.round_time(0) == T0 + HB // 11
    assert msgs.round_time(1) == T0 + 2 * HB // 11
    assert msgs.round_time(3 * R + 9) == T0 + 3 * HB + 10 * HB // 11


def test_flood_reaches_every_subscriber_at_bfs_depth():
    net, st = settled_state()
    msgs = ob.Msgs(net.n, 1, 8, R, T0, HB)
    g0 = 3 * R + 2                     # tick 3, after its control rounds settled
    first0 = st.first.copy()
    msgs.publish(st, 7, 0, 5, 0, g0)
    run_rounds(st, msgs, g0, g0 + R - 2)
    dist = mesh_bfs(net, st, 0, 5)
    assert (dist >= 0).all(), "mesh graph is connected"
    assert dist.max() <= R - 3
    slot = 7 % 8
    assert np.array_equal(msgs.seen[slot].astype(np.int64), g0 + dist)
    arrivals, firsts, dups, gray = msgs.stats
    assert firsts == net.n - 1 and gray == 0
    assert arrivals == firsts + dups
    # first-delivery credit: exactly one edge per non-origin receiver (markFirst)
    assert (st.first - first0).sum() == net.n - 1
    # expected arrivals: each peer forwards to its mesh minus the sender and the origin
    m = (st.tflags[0] & _abi.TF_MESH) != 0
    # the sender of j's first delivery is its lowest-index parent at dist-1
    exp = 0
    sender = np.full(net.n, -1)
    for i in range(net.n):
        if i == 5:
            continue
        b, e = int(net.row_ptr[i]), int(net.row_ptr[i + 1])
        cand = [int(net.col[x]) for x in range(b, e)
                if dist[int(net.col[x])] == dist[i] - 1 and m[st.rev[x]]]
        sender[i] = min(cand)          # lowest receiving edge == lowest sender index
    for j in range(net.n):
        for e in range(int(net.row_ptr[j]), int(net.row_ptr[j + 1])):
            i = int(net.col[e])
            if m[e] and i != 5 and i != sender[j]:
                exp += 1
    assert arrivals == exp


def test_first_delivery_credit_goes_to_lowest_sender():
    net, st = settled_state()
    msgs = ob.Msgs(net.n, 1, 4, R, T0, HB)
    g0 = 3 * R + 2
    first0 = st.first.copy()
    msgs.publish(st, 1, 0, 0, 0, g0)
    run_rounds(st, msgs, g0, g0 + R - 2)
    dist = mesh_bfs(net, st, 0, 0)
    m = (st.tflags[0] & _abi.TF_MESH) != 0
    d = st.first[0] - first0[0]
    for i in range(1, net.n):
        b, e = int(net.row_ptr[i]), int(net.row_ptr[i + 1])
        credited = [x for x in range(b, e) if d[x] != 0]
        assert len(credited) == 1
        parents = [x for x in range(b, e) if dist[int(net.col[x])] == dist[i] - 1 and m[st.rev[x]]]
        assert credited[0] == min(parents)


def test_duplicates_credit_mesh_deliveries_within_window():
    """markDuplicateMessageDelivery (score.go:951-981): within the window every
    mesh arrival counts; with a zero window only same-round duplicates do."""
    for window, exact in ((10 * Second, True), (0, False)):
        net, st = settled_state(window=window)
        msgs = ob.Msgs(net.n, 1, 4, R, T0, HB)
        g0 = 3 * R + 2
        meshd0 = st.meshd.copy()
        msgs.publish(st, 3, 0, 11, 0, g0)
        run_rounds(st, msgs, g0, g0 + R - 2)
        arrivals, firsts, dups, gray = msgs.stats
        credited = (st.meshd - meshd0).sum()
        if exact:
            assert credited == arrivals
        else:
            assert firsts <= credited < arrivals


def test_invalid_message_penalises_first_hop_only():
    """RejectMessage(ValidationFailed) -> markInvalidMessageDelivery; the
    rejected message is not forwarded (pubsub.go validation pipeline)."""
    net, st = settled_state()
    msgs = ob.Msgs(net.n, 1, 4, R, T0, HB)
    g0 = 3 * R + 2
    inv0 = st.invalid.copy()
    origin = 9
    msgs.publish(st, 0, 0, origin, 1, g0)
    run_rounds(st, msgs, g0, g0 + 4)
    m = (st.tflags[0] & _abi.TF_MESH) != 0
    b, e = int(net.row_ptr[origin]), int(net.row_ptr[origin + 1])
    hop1 = {int(net.col[x]) for x in range(b, e) if m[x]}
    seen = np.nonzero(msgs.seen[0] != ob.UNSEEN)[0]
    assert set(seen.tolist()) == hop1 | {origin}
    d = st.invalid[0] - inv0[0]
    assert d.sum() == len(hop1)
    assert (d[d != 0] == 1).all()
    assert (net.col[np.nonzero(d)[0]] == origin).all()


def test_graylisted_sender_is_ignored():
    """AcceptFrom (gossipsub.go:598-609): RPCs from peers scored below the
    graylist threshold are dropped before any processing."""
    net, st = settled_state()
    msgs = ob.Msgs(net.n, 1, 4, R, T0, HB)
    g0 = 3 * R + 2
    origin = 4
    st.score[net.col == origin] = -1000.0
    msgs.publish(st, 0, 0, origin, 0, g0)
    run_rounds(st, msgs, g0, g0 + 4)
    m = (st.tflags[0] & _abi.TF_MESH) != 0
    b, e = int(net.row_ptr[origin]), int(net.row_ptr[origin + 1])
    assert msgs.stats[3] == int(m[b:e].sum())
    assert msgs.stats[0] == 0
    assert (msgs.seen[0] == ob.UNSEEN).sum() == net.n - 1


def test_lastput_tracks_newest_mcache_put_per_topic():
    net, st = settled_state(T=2)
    msgs = ob.Msgs(net.n, 2, 8, R, T0, HB)
    g0 = 3 * R + 2
    msgs.publish(st, 0, 1, 3, 0, g0)
    run_rounds(st, msgs, g0, g0 + R - 2)
    assert (msgs.lastput[1] == 3).all()
    assert (msgs.lastput[0] == -1).all()


# ---- GPU parity -------------------------------------------------------------------

def _schedule(rng, ticks, T, R, rate, inv_frac, n):
    """Poisson publications per (round, topic): {round: [(id, topic, origin, invalid)]}."""
    sched, mid = {}, 0
    for k in ticks:
        for r in range(R):
            g = k * R + r
            batch = []
            for t in range(T):
                for _ in range(rng.poisson(rate / R)):
                    batch.append((mid, t, int(rng.integers(0, n)), int(rng.random() < inv_frac)))
                    mid += 1
            if batch:
                sched[g] = batch
    return sched


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,T,ticks,rate,inv_frac,retained,ring,send_variant", [
    (1500, 16, 2, [1, 2, 3, 4], 6, 0.1, 0.0, 256, 3),       # default: topic-major delivery
    (3000, 32, 3, [14, 15, 16], 12, 0.05, 0.03, 512, 3),    # clearBackoff tick
    (1500, 24, 2, [1, 2, 3, 4], 6, 0.1, 0.02, 256, 3),
    (1200, 16, 2, [1, 2], 200, 0.1, 0.02, 1024, 3),         # > 64 active slots a topic: passes, layers
    (1200, 16, 2, [1, 2], 200, 0.1, 0.02, 1024, 36),        # the same, blocks the same per topic
    (3000, 32, 10, [1, 2, 3], 12, 0.05, 0.02, 512, 3),      # 10 topics
])
def test_rounds_bit_exact(require_gpu, n, k, T, ticks, rate, inv_frac, retained, ring, send_variant):
    from fixtures import beacon_params, beacon_topic, synthetic_state
    from gsim.engine import Engine, random_regular
    from test_heartbeat import assert_same
    rng = np.random.default_rng(n + k)
    params = beacon_params(T)
    # a short duplicate window on one topic: only near-simultaneous copies count
    params.Topics["topic01"] = beacon_topic(MeshMessageDeliveriesWindow=150 * 10**6)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-100, PublishThreshold=-200, GraylistThreshold=-300)
    net = random_regular(n, k, seed=n, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    # some retained (disconnected) peers and heavy behaviour penalties: graylisted senders
    r = rng.random(net.e)
    st.estate[r < retained] = _abi.ES_TRACKED
    st.expire[r < retained] = tick_time(0) + rng.integers(1, 5, int((r < retained).sum())) * Second
    st.bp[rng.random(net.e) < 0.02] = 40.0
    msgs = ob.Msgs(n, T, ring, R, T0, HB)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    eng.msgs_init(ring, R, T0, HB)
    eng.set_kernel_variant(2, int(str(send_variant)[0]))
    if send_variant == 36:
        eng.set_kernel_variant(6, 1)
    sched = _schedule(rng, ticks, T, R, rate, inv_frac, n)
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
        seen = eng.read(_abi.F_SEEN)
        assert np.array_equal(seen, msgs.seen), f"seen-set differs at tick {kk}: {(seen != msgs.seen).sum()} cells"
        lp, want = eng.read(_abi.F_LASTPUT).ravel(), np.asarray(msgs.lastput).ravel()
        bad = np.nonzero(lp != want)[0]
        assert len(bad) == 0, f"lastput differs at tick {kk}: {len(bad)} entries, e.g. {[(int(b), int(lp[b]), int(want[b])) for b in bad[:4]]}"
        gpu = ob.NetState(net, params, thresholds=th, gossip=gp)
        gpu.pull_from_engine(eng)
        assert_same(st, gpu)
    assert msgs.stats[1] > n and msgs.stats[2] > n and msgs.stats[3] > 0
    eng.close()
