"""Validation latency and near-first crediting:
async validation windows (validation.go:246-407) with pending-duplicate
crediting (score.go:719-725, 806-811).

A message carries a validation latency of L rounds (gsim_msg.vdelay) at every
receiver.  A receiver that first sees it in round g marks it seen and fulfils
its IWANT promises then (ValidateMessage, gossip_tracer.go:163-168); its
verdict lands at the start of round g + L: DeliverMessage's
markFirstMessageDelivery for the first sender, markDuplicateMessageDelivery
with validated zero — so no window check — for every peer whose copy arrived
meanwhile (drec.peers), or RejectMessage's penalty for all of them; the
mcache.Put and forwarding follow (forwarded in round g + L + 1).  Copies
arriving from round g + L on are duplicates validated at round g + L.

CPU part: properties of the oracle's restatement against its own L = 0 run on
a fixed mesh (no heartbeat): every first reception is L rounds later per hop,
and the set of credited copies — hence every counter — is the same for a
window that credits every duplicate and for one that credits only same-round
copies.  GPU part: the engine bit-exact against the oracle through ticks with
gossip, every verdict, churn and the trace, for latencies 0-3 mixed."""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.engine import Engine, random_regular
from gsim.params import GossipSubParams, PeerScoreThresholds, Second
from gsim.presets import beacon_params, beacon_topic
from test_delivery import R, T0
from test_heartbeat import tick_time

TH = PeerScoreThresholds(GossipThreshold=-2000, PublishThreshold=-4000, GraylistThreshold=-8000)
GP = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)


def _params(T, window):
    p = beacon_params(T)
    for t in range(T):
        p.Topics[f"topic{t:02d}"] = beacon_topic(MeshMessageDeliveriesWindow=window)
    return p


def _oracle_run(L, verdict, window, seed=5):
    """One message from peer 0 on a fixed mesh, rounds only (no heartbeat, so
    no mesh change): the oracle's seen rounds and score counters."""
    from fixtures import synthetic_state
    net = random_regular(400, 10, seed=seed, n_topics=1)
    params = _params(1, window)
    st = ob.NetState(net, params, thresholds=TH, gossip=GP)
    synthetic_state(st, np.random.default_rng(seed), tick_time(0), 0.7)
    st.first[:] = 0.0
    st.meshd[:] = 0.0
    st.invalid[:] = 0.0
    msgs = ob.Msgs(net.n, 1, 64, R, T0, Second)
    g0 = 3 * R + 2
    msgs.publish(st, 0, 0, 0, verdict, g0, vdelay=L)
    for g in range(g0, g0 + 12 * (L + 1) + 2):
        msgs.round(st, g)
    return msgs.seen[0].astype(np.int64), st.first.copy(), st.meshd.copy(), st.invalid.copy(), g0


@pytest.mark.parametrize("L", [1, 3])
@pytest.mark.parametrize("window", [3600 * Second, 1])
def test_oracle_latency_delays_each_hop(L, window):
    s0, f0, m0, i0, g0 = _oracle_run(0, _abi.VERDICT_ACCEPT, window)
    sL, fL, mL, iL, _ = _oracle_run(L, _abi.VERDICT_ACCEPT, window)
    reached = s0 != _abi.UNSEEN
    assert reached.sum() > 300
    assert np.array_equal(reached, sL != _abi.UNSEEN)
    # hop h: seen at g0 + h without latency, validated at g0 + h (L + 1) with it
    assert np.array_equal(sL[reached] - g0, (s0[reached] - g0) * (L + 1))
    # the same first senders and the same credited copies
    assert np.array_equal(f0, fL) and f0.sum() > 300
    assert np.array_equal(m0, mL) and m0.sum() > 0
    assert not i0.any() and not iL.any()


def test_oracle_latency_reject_and_ignore():
    """A rejected message penalises its first copy and every copy that arrived
    while it was validated; an ignored one changes nothing."""
    for verdict in (_abi.VERDICT_REJECT, _abi.VERDICT_IGNORE):
        s0, f0, m0, i0, _ = _oracle_run(0, verdict, 3600 * Second)
        sL, fL, mL, iL, g0 = _oracle_run(2, verdict, 3600 * Second)
        assert np.array_equal(i0, iL)
        assert not fL.any() and not mL.any()
        assert (iL.sum() > 0) == (verdict == _abi.VERDICT_REJECT)
        # not forwarded: only the origin's mesh sees it, L rounds later validated
        recv = (s0 != _abi.UNSEEN) & (s0 != g0)
        assert recv.sum() > 0 and np.array_equal(sL != _abi.UNSEEN, s0 != _abi.UNSEEN)
        assert np.array_equal(sL[recv], s0[recv] + 2) and sL[0] == g0


@pytest.mark.gpu
def test_publish_rejects_bad_vdelay(require_gpu):
    eng = Engine(beacon_params(1), TH, gossip=GP)
    try:
        eng.load_graph(random_regular(200, 8, seed=3, n_topics=1))
        eng.msgs_init(64, R, T0, Second)
        with pytest.raises(Exception, match="vdelay"):
            eng.publish([(1, 0, 0, 0, _abi.MAX_VDELAY + 1)], 0)
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("window,trace", [(5 * 60 * Second, None), (100_000_000, (0, 700))])
def test_validation_latency_bit_exact(require_gpu, window, trace):
    from fixtures import synthetic_state
    from tickrun import run_parity, subscribed_schedule
    rng = np.random.default_rng(41)
    n, k, T = 1500, 16, 3
    params = _params(T, window)
    net = random_regular(n, k, seed=43, n_topics=T)
    st = ob.NetState(net, params, thresholds=TH, gossip=GP)
    synthetic_state(st, rng, tick_time(0), 0.6)
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.0, verdicts=(0.7, 0.1, 0.1, 0.05, 0.05),
                                vdelays=(0, 1, 2, 3))
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 40, replace=False)]
    churn = {3: [(down, False)], 5: [(down, True)]}
    msgs, gstats = run_parity(net, params, TH, GP, st, ticks, sched, ring=512, churn=churn, trace=trace)
    assert msgs.stats[1] > 0 and gstats["iwant_ids"] > 0, "first deliveries and IWANTs happened"


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("shards", [2, 3])
def test_validation_latency_sharded_bit_exact(require_gpu, shards):
    """Validation latency on a graph-sharded network (copy push): pending
    duplicates of copies pushed from other shards queue at the receiver's
    shard, completions forward from the owner's shard, and the ghosts'
    holder rounds carry the completion round — bit-exact against the oracle
    with every verdict, gossip and churn."""
    from fixtures import synthetic_state
    from gsim.shard import ShardedEngine
    from tickrun import SEED, run_parity, subscribed_schedule
    rng = np.random.default_rng(43 + shards)
    n, k, T = 1500, 16, 3
    params = _params(T, 5 * 60 * Second)
    net = random_regular(n, k, seed=47, n_topics=T)
    st = ob.NetState(net, params, thresholds=TH, gossip=GP)
    synthetic_state(st, rng, tick_time(0), 0.6)
    eng = ShardedEngine(params, TH, gossip=GP, shards=shards)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.0, verdicts=(0.7, 0.1, 0.1, 0.05, 0.05),
                                vdelays=(0, 1, 2, 3))
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 40, replace=False)]
    churn = {3: [(down, False)], 5: [(down, True)]}
    msgs, gstats = run_parity(net, params, TH, GP, st, ticks, sched, ring=512, churn=churn, eng=eng)
    assert msgs.stats[1] > 0 and gstats["iwant_ids"] > 0, "first deliveries and IWANTs happened"


# RejectMessage reasons of each verdict (tracer.go:28-38, oracle.h ORC_REJECT_*)
_REASON = {_abi.VERDICT_REJECT: 8, _abi.VERDICT_IGNORE: 9, _abi.VERDICT_THROTTLE: 7}


@pytest.mark.parametrize("L", [0, 2])
def test_latency_follows_the_pinned_score_tracer(L):
    """The network oracle's crediting equals the KAT-pinned per-observer score
    tracer (oracle.c's delivery records, score_test.go) driven by the same
    copies in Go's call order: ValidateMessage at the first reception,
    DuplicateMessage at every later copy, Deliver/RejectMessage when the
    validation completes — for every receiver, with a window (150 ms) that
    credits some later duplicates and not others."""
    from fixtures import synthetic_state
    net = random_regular(300, 10, seed=9, n_topics=1)
    params = _params(1, 150_000_000)
    lib = ob.load()

    def state():
        st = ob.NetState(net, params, thresholds=TH, gossip=GP)
        synthetic_state(st, np.random.default_rng(9), tick_time(0), 0.7)
        for f in (st.first, st.meshd, st.invalid):
            f[:] = 0.0
        return st

    st, replay = state(), state()
    assert np.array_equal(st.tflags, replay.tflags)
    msgs = ob.Msgs(net.n, 1, 64, R, T0, Second)
    msgs.log()
    g0 = 2 * R + 3
    pubs = {g0: (0, 5, _abi.VERDICT_ACCEPT), g0 + 1: (1, 77, _abi.VERDICT_REJECT),
            g0 + 2: (2, 150, _abi.VERDICT_ACCEPT), g0 + 4: (3, 201, _abi.VERDICT_IGNORE),
            g0 + 5: (4, 260, _abi.VERDICT_THROTTLE), g0 + 6: (5, 33, _abi.VERDICT_ACCEPT)}
    verdict = {mid: v for (mid, _, v) in pubs.values()}
    for g in range(g0, g0 + 40):
        if g in pubs:
            mid, origin, v = pubs[g]
            msgs.publish(st, mid, 0, origin, v, g, vdelay=L)
        msgs.round(st, g)
    ev = msgs.events()
    seen = ev[(ev["kind"] == ob.EV_SEEN) & (ev["b"] != 0xFFFFFFFF)]
    assert len(seen) > 1000

    def edge(a, b):
        lo, hi = int(net.row_ptr[a]), int(net.row_ptr[a + 1])
        return lo + int(np.nonzero(net.col[lo:hi] == b)[0][0])

    # (round, phase, receiver, ...): completions open a round (phase 0; with
    # no latency right after the first reception, 1.5), then first
    # receptions (1), then duplicates (2)
    acts = []
    for e in seen:
        a, b, g, mid = int(e["a"]), int(e["b"]), int(e["g"]), int(e["mid"])
        if int(e["x"]):
            acts.append((g - L, 1, a, b, mid, "validate"))
            acts.append((g, 0 if L else 1.5, a, b, mid, "complete"))
        else:
            acts.append((g, 2, a, b, mid, "duplicate"))
    acts.sort(key=lambda x: (x[0], x[1], x[2], x[4], x[3]))
    v = replay.view()
    drecs = {}
    try:
        for (g, _, a, b, mid, what) in acts:
            d = drecs.setdefault(a, lib.orc_drecs_new(int(params.SeenMsgTTL)))
            now = msgs.round_time(g)
            if what == "validate":
                lib.orc_validate_message(v, d, mid, now)
            elif what == "duplicate":
                lib.orc_duplicate_message(v, d, edge(a, b), mid, 0, now)
            elif verdict[mid] == _abi.VERDICT_ACCEPT:
                lib.orc_deliver_message(v, d, edge(a, b), mid, 0, now)
            else:
                lib.orc_reject_message(v, d, edge(a, b), mid, 0, _REASON[verdict[mid]], now)
    finally:
        for d in drecs.values():
            lib.orc_drecs_free(d)
    for f in ("first", "meshd", "invalid"):
        assert np.array_equal(getattr(st, f), getattr(replay, f)), f
    assert st.first.sum() > 0 and st.meshd.sum() > 0 and st.invalid.sum() > 0
