"""Gossip: emitGossip IHAVE -> handleIHave IWANT -> handleIWant response,
and the gossip tracer's IWANT promises with the broken-promise P7 penalty
(gossipsub.go:630-739, 1620-1625, 1711-1775; gossip_tracer.go:48-141;
mcache.go:55-104).

CPU part: behavioural invariants of the oracle restatement, mirroring what
the reference's tests assert — a peer the mesh cannot reach still gets a
message through IHAVE/IWANT (gossipsub_test.go TestGossipsubGossip*), and a
peer that advertises but never answers IWANT is penalised through P7
(gossipsub_spam_test.go:134-286, TestGossipsubAttackSpamIWANT).  GPU part:
the engine against the oracle, bit-exact, across heartbeats with gossip.
"""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second
from test_delivery import R, T0, delivery_params
from test_heartbeat import SEED, tick_time

TH = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-60, GraylistThreshold=-100)


def gossip_net(n=400, k=16, T=1):
    from gsim.engine import random_regular
    net = random_regular(n, k, seed=3, n_topics=T)
    st = ob.NetState(net, delivery_params(T), thresholds=TH, gossip=GossipSubParams(D=6, Dlo=5, Dhi=12))
    return net, st


def run_tick(st, msgs, kk, sched=None, isolate=None):
    """One BSP tick of the oracle: refresh, broken-promise penalties, score,
    heartbeat + emitGossip, R rounds (control + IHAVE/IWANT inside)."""
    lib = ob.load()
    v = st.view()
    now = tick_time(kk)
    lib.orc_refresh_scores(v, now)
    msgs.penalties(st, now)
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    msgs.heartbeat(st, kk, now, SEED)
    for g in range(kk * R, kk * R + R):
        if isolate is not None:
            isolate()
        for (mid, t, o, inv) in (sched or {}).get(g, []):
            msgs.publish(st, mid, t, o, inv, g)
        msgs.round(st, g)


def cut_mesh(net, st, p):
    """Remove peer p from every mesh (both directions), as after churn."""
    rev = st.rev
    for e in range(int(net.row_ptr[p]), int(net.row_ptr[p + 1])):
        st.tflags[:, e] &= ~np.uint8(_abi.TF_MESH)
        st.tflags[:, rev[e]] &= ~np.uint8(_abi.TF_MESH)
        st.ctl[:, :, e] = 0
        st.ctl[:, :, rev[e]] = 0


def test_gossip_recovers_message_the_mesh_missed():
    net, st = gossip_net()
    msgs = ob.Msgs(net.n, 1, 64, R, T0, tick_time(1) - tick_time(0))
    for kk in range(1, 4):
        run_tick(st, msgs, kk)
    p = 7
    k = 4
    # tick 4: p is outside every mesh while a message floods the network
    cut = lambda: cut_mesh(net, st, p)  # noqa: E731
    run_tick(st, msgs, k, sched={k * R + 1: [(5, 0, 100, 0)]}, isolate=cut)
    slot = 5 % 64
    assert msgs.seen[slot, p] == ob.UNSEEN, "the mesh cannot reach p"
    assert (msgs.seen[slot] != ob.UNSEEN).sum() == net.n - 1
    first0 = st.first.copy()
    run_tick(st, msgs, k + 1)
    # IHAVE at heartbeat 5, IWANT in round 0, response in round 1, arrival in round 2
    assert msgs.seen[slot, p] == (k + 1) * R + 2
    b, en = int(net.row_ptr[p]), int(net.row_ptr[p + 1])
    credited = [e for e in range(b, en) if st.first[0, e] != first0[0, e]]
    assert len(credited) == 1, "markFirstMessageDelivery for the responding peer only"


def test_ignored_iwant_breaks_promise_and_penalises():
    net, st = gossip_net()
    beh = np.full(net.n, ob.ORC_BEHAVE_IGNORE_IWANT, np.uint8)
    p = 7
    beh[p] = 0
    msgs = ob.Msgs(net.n, 1, 64, R, T0, tick_time(1) - tick_time(0), behaviour=beh)
    for kk in range(1, 4):
        run_tick(st, msgs, kk)
    k = 4
    cut = lambda: cut_mesh(net, st, p)  # noqa: E731
    run_tick(st, msgs, k, sched={k * R + 1: [(5, 0, 100, 0)]}, isolate=cut)
    b, en = int(net.row_ptr[p]), int(net.row_ptr[p + 1])
    bp_hist = []
    for kk in range(k + 1, k + 7):
        run_tick(st, msgs, kk)
        bp_hist.append(st.bp[b:en].copy())
    assert msgs.seen[5 % 64, p] == ob.UNSEEN, "nobody answers p's IWANT"
    # the first promise (heartbeat 5, expiry = round 0 of tick 5 + 3 s) is
    # still pending at heartbeat 8 and broken at heartbeat 9
    for h in range(4):
        assert (bp_hist[h] == 0).all(), f"no penalty before heartbeat 9 (tick {k + 1 + h})"
    jumped = np.nonzero(bp_hist[4] >= 1.0)[0]
    assert len(jumped) >= 1, "AddPenalty(peer, brokenPromises) on the advertiser p asked"


# ---- GPU parity -------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("n,k,T,nticks,rate,ignore_frac,ring", [
    (1200, 16, 2, 8, 8, 0.1, 256),
    (2000, 32, 3, 7, 10, 0.3, 512),
    (800, 24, 40, 7, 1, 0.2, 2048),      # T > 32 with two observers per wavefront (topics gl and gl+32)
    (1000, 16, 20, 7, 1, 0.2, 1024),     # four observers per wavefront, T > 16 (topics gl and gl+16)
])
def test_gossip_rounds_bit_exact(require_gpu, n, k, T, nticks, rate, ignore_frac, ring):
    """Heartbeats with emitGossip, IHAVE/IWANT in control rounds 0/1, the
    responses in round 2, promises breaking four heartbeats later (P7): every
    state array, the seen-set and the delivery totals bit-exact per tick."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import Engine, random_regular
    from test_delivery import _schedule
    from test_heartbeat import assert_same
    rng = np.random.default_rng(n * 7 + k)
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-50, GraylistThreshold=-300)
    net = random_regular(n, k, seed=n + 1, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    st.bp[rng.random(net.e) < 0.03] = 12.0          # some low scores: gossip and IWANT gates bite
    beh = (rng.random(n) < ignore_frac).astype(np.uint8) * ob.ORC_BEHAVE_IGNORE_IWANT
    msgs = ob.Msgs(n, T, ring, R, T0, Second, behaviour=beh)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    eng.msgs_init(ring, R, T0, Second)
    eng.set_peer_behaviour(beh)
    ticks = list(range(1, nticks + 1))
    sched = _schedule(rng, ticks, T, R, rate, 0.05, n)
    lib = ob.load()
    bp0 = None
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
        assert np.array_equal(eng.read(_abi.F_LASTPUT), msgs.lastput)
        gpu = ob.NetState(net, params, thresholds=th, gossip=gp)
        gpu.pull_from_engine(eng)
        assert_same(st, gpu)
        if kk == 2:
            bp0 = st.bp.copy()
    # gossip did work: messages first delivered in round 2 of a tick by IWANT
    # responses, and broken promises raised some behaviour penalties
    assert (msgs.seen % R == 2).any()
    assert (st.bp > bp0 * 0.5 + 0.5).any()
    eng.close()


@pytest.mark.gpu
def test_iwant_response_queue_overflow_is_reported(require_gpu):
    """A response queue smaller than the IWANT traffic: the overflow is
    reported by the next heartbeat and by gsim_msg_stats (GSIM_ERANGE), and
    nothing past the queue is read or written."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import Engine, GsimError, random_regular
    from test_delivery import _schedule
    rng = np.random.default_rng(77)
    n, k, T = 1200, 16, 1
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-50, GraylistThreshold=-300)
    net = random_regular(n, k, seed=5, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    eng.msgs_init(256, R, T0, Second, max_arrivals=4)
    ticks = list(range(1, 6))
    sched = _schedule(rng, ticks, T, R, 10, 0.0, n)
    stopped = None
    for kk in ticks:
        now = tick_time(kk)
        eng.refresh_scores(now)
        try:
            eng.heartbeat(kk, now)
        except GsimError as ex:          # the previous tick overflowed: stop before running on
            stopped = (kk, ex.rc)
            break
        for g in range(kk * R, kk * R + R):
            if g in sched:
                eng.publish(sched[g], g)
            eng.round(g)
    assert stopped is not None and stopped[1] == _abi.GSIM_ERANGE
    with pytest.raises(GsimError) as ei:
        eng.msg_stats()
    assert ei.value.rc == _abi.GSIM_ERANGE
    assert eng.gossip_stats()["iwant_responses"] > 4
    eng.close()


def _gossip_window_run(max_ihave_length, ring=1024, n=1200, T=8, rate=10, ticks=5):
    """Every topic busy: several messages per topic in each gossip window."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import Engine, random_regular
    from test_delivery import _schedule
    rng = np.random.default_rng(4242)
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, MaxIHaveLength=max_ihave_length)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-50, GraylistThreshold=-300)
    net = random_regular(n, 16, seed=n + 3, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / 16)
    sched = _schedule(rng, list(range(1, ticks + 1)), T, R, rate, 0.0, n)
    return net, params, th, gp, st, sched


@pytest.mark.gpu
def test_ring_larger_than_max_ihave_length_bit_exact(require_gpu):
    """A ring larger than MaxIHaveLength (gsim_msgs_init accepts it): the
    gossip window holds more ids than MaxIHaveLength in all, but no topic's
    window and no IWANT list exceeds it, so no truncation applies
    (gossipsub.go:679-690, 1766-1771) and the device is bit-exact with the
    oracle, which implements the truncations."""
    from tickrun import run_parity
    net, params, th, gp, st, sched = _gossip_window_run(max_ihave_length=60)
    msgs, gs = run_parity(net, params, th, gp, st, list(range(1, 6)), sched, ring=1024)
    assert gs["iwant_ids"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("max_ihave_length", [4, 25])
def test_max_ihave_length_truncations_bit_exact(require_gpu, max_ihave_length):
    """Gossip windows over MaxIHaveLength: an advertiser sends each target a
    random MaxIHaveLength-subset of a topic's window (emitGossip,
    gossipsub.go:1763-1772) and a receiver asks for at most MaxIHaveLength
    ids (handleIHave, gossipsub.go:679-690), with the promise among them.
    k_ihave_pairs against the oracle's truncations, bit-exact per tick."""
    from tickrun import run_parity
    net, params, th, gp, st, sched = _gossip_window_run(max_ihave_length=max_ihave_length)
    msgs, gs = run_parity(net, params, th, gp, st, list(range(1, 6)), sched, ring=1024)
    assert gs["iwant_ids"] > 0 and gs["iwant_responses"] > 0


def _retransmission_case(retransmission):
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import subscribed_schedule
    rng = np.random.default_rng(3131 + retransmission)
    n, k, T = 800, 16, 2
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, GossipRetransmission=retransmission)
    th = PeerScoreThresholds(GossipThreshold=-20000, PublishThreshold=-50000, GraylistThreshold=-80000)
    net = random_regular(n, k, seed=n + 9, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    ticks = list(range(1, 8))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.0, verdicts=(0.5, 0.0, 0.0, 0.0, 0.5))
    return net, params, th, gp, st, ticks, sched


@pytest.mark.parametrize("retransmission", [1, 2])
def test_retransmission_case_refuses_serves_in_the_oracle(retransmission):
    """The GPU case below is sensitive: in the oracle some (message, peer)
    pairs are asked for more than GossipRetransmission times, and refused."""
    net, params, th, gp, st, ticks, sched = _retransmission_case(retransmission)
    msgs = ob.Msgs(net.n, st.T, 512, R, T0, Second)
    msgs.log()
    lib = ob.load()
    refused = 0
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
        ev = msgs.events()
        refused += int(((ev["kind"] == ob.EV_SERVE) & (ev["x"] > retransmission)).sum())
    assert refused > 0


@pytest.mark.gpu
@pytest.mark.parametrize("retransmission", [1, 2])
def test_gossip_retransmission_limits_bad_signature_serves(require_gpu, retransmission):
    """mcache.GetForPeer's count (mcache.go:73-86, handleIWant
    gossipsub.go:712-715): a message with a bad signature is never marked
    seen by its receivers, so they keep asking its origin; answers beyond
    GossipRetransmission per (message, peer) are refused.  Bit-exact with the
    oracle's peertx table."""
    from tickrun import run_parity
    net, params, th, gp, st, ticks, sched = _retransmission_case(retransmission)
    msgs, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=512)
    assert gs["iwant_responses"] > 0
