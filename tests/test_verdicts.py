"""Validation verdicts: accept / reject / ignore /
throttle / invalid signature, as the score tracer sees them
(score.go:693-827 ValidateMessage / RejectMessage / DuplicateMessage,
gossip_tracer.go:148-170, validation.go:282-290).

The reference's tests this follows:
  * gossipsub_test.go:1610-1695 TestGossipsubScoreValidatorEx — three fully
    connected hosts; host1's message is ignored, host2's rejected: host0's
    score of host1 stays 0, of host2 turns negative;
  * score_test.go:548-645 TestScoreRejectMessageDeliveries — ignored and
    throttled messages leave the score alone, a failed validation costs the
    sender -1 (InvalidMessageDeliveriesWeight -1, TopicWeight 1).

In the simulation a message carries one verdict for every receiver
(gsim_msg.verdict): only accepted copies are forwarded, so the origin is the
only sender of a non-accepted message.  CPU part: the oracle.  GPU part: the
engine bit-exact against it, and the same invariants read from the device.
"""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.engine import Network
from gsim.params import GossipSubParams, PeerScoreParams, PeerScoreThresholds, Second, TopicScoreParams
from test_delivery import R, T0
from test_heartbeat import SEED, tick_time

V = {"accept": _abi.VERDICT_ACCEPT, "reject": _abi.VERDICT_REJECT, "ignore": _abi.VERDICT_IGNORE,
     "throttle": _abi.VERDICT_THROTTLE, "signature": _abi.VERDICT_SIGNATURE}


def validator_ex():
    """gossipsub_test.go:1615-1635: the params and thresholds of the test."""
    params = PeerScoreParams(
        AppSpecificScore=lambda p: 0.0, DecayInterval=Second, DecayToZero=0.01,
        Topics={"test": TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second,
                                         InvalidMessageDeliveriesWeight=-1,
                                         InvalidMessageDeliveriesDecay=0.9999)})
    th = PeerScoreThresholds(GossipThreshold=-10, PublishThreshold=-100, GraylistThreshold=-10000)
    return params, th


def complete_net(n):
    """connectAll: every pair connected (rows in peer order), one topic joined by all."""
    cols = [[j for j in range(n) if j != i] for i in range(n)]
    row_ptr = np.zeros(n + 1, dtype=np.uint32)
    row_ptr[1:] = np.cumsum([len(c) for c in cols])
    col = np.array([j for c in cols for j in c], dtype=np.uint32)
    ip_ptr = np.arange(n + 1, dtype=np.uint32)
    return Network(n, row_ptr, col, np.zeros(len(col), np.uint8), np.ones(n, np.uint64),
                   ip_ptr, np.arange(n, dtype=np.uint32), n)


def record(net, observer, peer):
    """Index of observer's record about peer (the rev of the copy's edge in
    the sender's row, as the delivery kernels credit it)."""
    b, e = int(net.row_ptr[observer]), int(net.row_ptr[observer + 1])
    return b + int(np.nonzero(net.col[b:e] == peer)[0][0])


def run_oracle(net, params, th, gp, publications, ticks=(1, 2)):
    """publications: [(id, origin, verdict)] published in round 1 of the first tick."""
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    msgs = ob.Msgs(net.n, 1, 64, R, T0, Second)
    lib = ob.load()
    for kk in ticks:
        now = tick_time(kk)
        v = st.view()
        lib.orc_refresh_scores(v, now)
        msgs.penalties(st, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
        msgs.heartbeat(st, kk, now, SEED)
        for g in range(kk * R, kk * R + R):
            if kk == ticks[0] and g == kk * R + 1:
                for (mid, origin, vd) in publications:
                    msgs.publish(st, mid, 0, origin, vd, g)
            msgs.round(st, g)
    # the scores the next refresh sees
    now = tick_time(ticks[-1] + 1)
    v = st.view()
    lib.orc_refresh_scores(v, now)
    lib.orc_compute_scores(v)
    return st, msgs


def test_validator_ex_ignore_keeps_zero_reject_turns_negative():
    """TestGossipsubScoreValidatorEx: host1's message ignored, host2's rejected."""
    params, th = validator_ex()
    net = complete_net(3)
    st, msgs = run_oracle(net, params, th, GossipSubParams(),
                          [(1, 1, V["ignore"]), (2, 2, V["reject"])])
    assert st.score[record(net, 0, 1)] == 0.0, "ignored: no penalty"
    assert st.score[record(net, 0, 2)] < 0.0, "rejected: P4"
    # nobody forwarded either message: host0 got each from its origin only
    assert msgs.stats[2] == 0, "no duplicates: non-accepted messages are not forwarded"


@pytest.mark.parametrize("verdict,penalised,seen", [
    ("accept", False, True), ("ignore", False, True), ("throttle", False, True),
    ("reject", True, True), ("signature", True, False)])
def test_reject_message_deliveries(verdict, penalised, seen):
    """TestScoreRejectMessageDeliveries: throttled / ignored leave the score
    at 0, a failed validation (or a bad signature) costs P4 = -invalid^2;
    a bad signature is never marked seen (validation.go:282-290)."""
    params, th = validator_ex()
    net = complete_net(4)
    st, msgs = run_oracle(net, params, th, GossipSubParams(), [(5, 3, V[verdict])], ticks=(1,))
    for obs in range(3):
        r = record(net, obs, 3)
        inv = st.invalid[0, r]
        if penalised:
            # one invalid delivery decayed once by the refresh that scored it
            assert inv == pytest.approx(0.9999) and st.score[r] == pytest.approx(-(0.9999 ** 2))
        else:
            assert inv == 0.0 and st.score[r] == 0.0
        assert (msgs.seen[5 % 64, obs] != ob.UNSEEN) == seen
    # only accepted copies are forwarded: duplicates exist for those alone
    assert (msgs.stats[2] > 0) == (verdict in ("accept", "signature"))


# ---- GPU --------------------------------------------------------------------------


def _engine_parity(net, params, th, gp, sched, ticks, ring=64):
    from tickrun import run_parity
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    return run_parity(net, params, th, gp, st, ticks, sched, ring=ring)


@pytest.mark.gpu
def test_validator_ex_on_device(require_gpu):
    """The ValidatorEx scenario through the engine: bit-exact with the oracle
    every tick, then host0's scores of host1 (ignored) = 0, of host2
    (rejected) < 0, read from the device snapshot."""
    from gsim.engine import Engine
    params, th = validator_ex()
    gp = GossipSubParams()
    net = complete_net(3)
    sched = {R + 1: [(1, 0, 1, V["ignore"]), (2, 0, 2, V["reject"])]}
    _engine_parity(net, params, th, gp, sched, [1, 2])
    eng = Engine(params, th, gossip=gp)
    try:
        eng.load_graph(net)
        eng.set_seed(SEED)
        eng.msgs_init(64, R, T0, Second)
        for kk in (1, 2):
            eng.refresh_scores(tick_time(kk))
            eng.heartbeat(kk, tick_time(kk))
            for g in range(kk * R, kk * R + R):
                if g in sched:
                    eng.publish(sched[g], g)
                eng.round(g)
        eng.refresh_scores(tick_time(3))
        score = eng.read(_abi.F_SCORE)
        assert score[record(net, 0, 1)] == 0.0
        assert score[record(net, 0, 2)] < 0.0
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,T", [(1500, 16, 2), (2000, 32, 3)])
def test_mixed_verdicts_bit_exact(require_gpu, n, k, T):
    """Every verdict in one run (a fifth of the messages not accepted): the
    seen-set, delivery totals, mcache puts and every record bit-exact per
    tick with gossip, promises and control."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import run_parity, subscribed_schedule
    rng = np.random.default_rng(n + 3 * k)
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-100, GraylistThreshold=-300)
    net = random_regular(n, k, seed=n + 11, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 6.0, 0.0, verdicts=(0.8, 0.05, 0.05, 0.05, 0.05))
    kinds = {m[3] for b in sched.values() for m in b}
    assert kinds == set(V.values()), "every verdict appears"
    msgs, _ = run_parity(net, params, th, gp, st, ticks, sched, ring=512)
    assert msgs.stats[1] > n


@pytest.mark.gpu
def test_invalid_planes_skipped_while_zero_bit_exact(require_gpu):
    """The refresh reads no invalidMessageDeliveries plane while every counter
    is zero (engine.hip k_refresh_score, Handle::d_inv_live).  Rejected
    messages raise counters (ticks 1-2), a fast decay takes every one back to
    zero (ticks 3-8, the flag clears), counters written through the ABI and
    new rejections bring them back (ticks 9-11): every record bit-exact per
    tick on both sides of each transition."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import run_parity, subscribed_schedule
    n, k, T = 1500, 16, 2
    rng = np.random.default_rng(77)
    params = beacon_params(T)
    for tp in params.Topics.values():
        tp.InvalidMessageDeliveriesDecay = 0.2          # 1.0 -> below DecayToZero (0.01) in 3 ticks
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-100, GraylistThreshold=-300)
    net = random_regular(n, k, seed=91, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    st.invalid[...] = 0.0
    sched = {}
    for ticks, inv in (([1, 2], 0.3), (list(range(3, 11)), 0.0), ([11], 0.3)):
        sched.update(subscribed_schedule(rng, ticks, net, T, 6.0, inv))
    mid = 0
    for g in sorted(sched):                              # ids unique across the three parts
        sched[g] = [(mid + q,) + m[1:] for q, m in enumerate(sched[g])]
        mid += len(sched[g])
    seen_zero = []

    def after_heartbeat(kk, eng, st_, msgs):
        if kk == 8:
            seen_zero.append(eng.census()["nz_invalid"])
        if kk == 9:
            recs = rng.choice(net.e, 40, replace=False)
            st_.invalid[0, recs] = 2.5
            st_.invalid[T - 1, recs[:10]] = 0.75
            eng.write(_abi.F_INVALID, st_.invalid)

    msgs, _ = run_parity(net, params, th, gp, st, list(range(1, 12)), sched, ring=512,
                         after_heartbeat=after_heartbeat)
    assert seen_zero == [0], "every invalid counter back at zero before the ABI write"
    assert (st.invalid != 0).any(), "counters non-zero again at the end"
