"""Peer gater (peer_gater.go): WithPeerGater's
random-early-drop AcceptFrom over per-IP delivery statistics.

CPU part: PeerGaterParams.validate's table (peer_gater.go:57-90, the same
messages), NewPeerGaterParams / DefaultPeerGaterParams defaults
(peer_gater.go:19-28, 99-116), and TestPeerGater (peer_gater_test.go:11-121)
restated step by step on the oracle's gater (its deterministic draws: a
stream of Philox uniforms instead of math/rand).

GPU part: the engine's gater on a network with shared IPs, throttled
validations, churn and gossip, bit-exact against the oracle every tick
(every counter, lastThrottle, connected / expire, the drop count, and the
whole network state through the gated deliveries)."""
import ctypes

import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import (DefaultPeerGaterParams, Hour, Minute, NewPeerGaterParams, PeerGaterParams,
                         ScoreParameterDecay, Second)


# ---- CPU -------------------------------------------------------------------------------

@pytest.mark.parametrize("field,value,msg", [
    ("Threshold", 0.0, "invalid Threshold; must be > 0"),
    ("GlobalDecay", 0.0, "invalid GlobalDecay; must be between 0 and 1"),
    ("GlobalDecay", 1.0, "invalid GlobalDecay; must be between 0 and 1"),
    ("SourceDecay", 0.0, "invalid SourceDecay; must be between 0 and 1"),
    ("SourceDecay", 1.0, "invalid SourceDecay; must be between 0 and 1"),
    ("DecayInterval", Second - 1, "invalid DecayInterval; must be at least 1s"),
    ("DecayToZero", 0.0, "invalid DecayToZero; must be between 0 and 1"),
    ("DecayToZero", 1.0, "invalid DecayToZero; must be between 0 and 1"),
    ("Quiet", Second - 1, "invalud Quiet interval; must be at least 1s"),
    ("DuplicateWeight", 0.0, "invalid DuplicateWeight; must be > 0"),
    ("IgnoreWeight", 0.5, "invalid IgnoreWeight; must be >= 1"),
    ("RejectWeight", 0.5, "invalud RejectWeight; must be >= 1"),
])
def test_gater_params_validate(field, value, msg):
    """PeerGaterParams.validate (peer_gater.go:57-90), messages as in the reference."""
    p = NewPeerGaterParams(0.1, 0.9, 0.999)
    p.validate()
    assert ob.load().orc_gater_validate(ctypes.byref(p.to_c())) == 0
    setattr(p, field, value)
    with pytest.raises(ValueError, match=msg.replace("(", r"\(")):
        p.validate()
    assert ob.load().orc_gater_validate(ctypes.byref(p.to_c())) != 0


def test_gater_default_params():
    """NewPeerGaterParams / DefaultPeerGaterParams (peer_gater.go:19-28, 99-116)."""
    p = NewPeerGaterParams(0.1, 0.9, 0.999)
    assert (p.Threshold, p.GlobalDecay, p.SourceDecay) == (0.1, 0.9, 0.999)
    assert p.DecayToZero == 0.01 and p.DecayInterval == Second
    assert p.RetainStats == 6 * Hour and p.Quiet == Minute
    assert (p.DuplicateWeight, p.IgnoreWeight, p.RejectWeight) == (0.125, 1.0, 16.0)
    d = DefaultPeerGaterParams()
    assert d.Threshold == 0.33
    assert d.GlobalDecay == ScoreParameterDecay(2 * Minute)
    assert d.SourceDecay == ScoreParameterDecay(Hour)


def _two_peer_state(gater):
    """Router 0 connected to peer A = 1 (IP "1.2.3.4"), the gater on."""
    from fixtures import beacon_params
    from gsim.engine import Network
    row_ptr = np.array([0, 1, 2], dtype=np.uint32)
    col = np.array([1, 0], dtype=np.uint32)
    net = Network(2, row_ptr, col, np.array([1, 0], dtype=np.uint8), np.ones(2, dtype=np.uint64),
                  np.array([0, 1, 2], dtype=np.uint32), np.array([0, 7], dtype=np.uint32), 8)
    st = ob.NetState(net, beacon_params(1))
    st.estate[...] = _abi.ES_TRACKED | _abi.ES_CONNECTED
    st.enable_gater(gater)
    return st


def test_peer_gater_restated():
    """TestPeerGater (peer_gater_test.go:11-121), step by step on the oracle's
    gater: AcceptFrom is AcceptAll until validation throttles, turns into
    AcceptControl once the peer's IP has a bad record, accepts again after
    deliveries and decays back to AcceptAll; RemovePeer keeps the IP's stats
    until RetainStats has passed."""
    lib = ob.load()
    st = _two_peer_state(NewPeerGaterParams(0.1, 0.9, 0.999))
    now = 1000 * Second
    seed = 0xC0FFEE
    draws = {"g": 0}

    def accept_from():
        v = st.view()
        lib.orc_gater_round_begin(v, now)
        draws["g"] += 1
        return lib.orc_gater_accept(v, seed, draws["g"], 0, 0, 0) == 1      # router 0, its edge 0 (to A)

    def events(*kinds, n=1):
        v = st.view()
        for _ in range(n):
            for k in kinds:
                lib.orc_gater_event(v, 0, 0, 0, k)
        lib.orc_gater_round_end(v, now)

    assert accept_from()                                    # pg.AddPeer(peerA): nothing throttled yet
    events(st.GATE_VALIDATE)
    assert accept_from()                                    # throttle == 0
    events(st.GATE_THROTTLE)                                # RejectValidationQueueFull
    assert accept_from()                                    # no stats for A's IP: total == 0
    events(st.GATE_THROTTLE)                                # RejectValidationThrottled
    assert accept_from()
    events(st.GATE_IGNORE, st.GATE_REJECT, n=100)
    assert any(not accept_from() for _ in range(1000)), "expected AcceptControl"
    s = st.gater_read()
    assert (s["validate"][0], s["throttle"][0], s["last"][0]) == (1.0, 2.0, now)
    assert list(s["counters"][:, 0]) == [0.0, 0.0, 100.0, 100.0]
    events(st.GATE_DELIVER, n=100)
    assert any(accept_from() for _ in range(1000)), "expected to accept at least once"
    for _ in range(100):
        st.gater_decay(now)
    assert accept_from()                                    # validate / throttle decayed to zero
    s = st.gater_read()
    assert s["throttle"][0] == 0.0 and s["validate"][0] == 0.0
    lib.orc_gater_connection(st.view(), 0, 0, now)          # pg.RemovePeer(peerA)
    s = st.gater_read()
    assert s["connected"][0] == 0 and s["expire"][0] == now + 6 * Hour
    assert s["counters"][0, 0] > 0, "expected to still have a stat record for peerA's ip"
    st.gater_decay(now + 6 * Hour - 1)                      # retained, not decayed (no connected peer)
    assert st.gater_read()["counters"][0, 0] == s["counters"][0, 0]
    st.gater_decay(now + 6 * Hour + 1)                      # expired: deleted
    assert not st.gater_read()["counters"][:, 0].any(), "still have a stat record for peerA's ip"


def test_gater_drop_rate_follows_goodput():
    """The drop probability is 1 - (1 + deliver) / (1 + weighted total)
    (peer_gater.go:346-362): over many draws the oracle's Philox uniforms hit
    it within sampling error."""
    lib = ob.load()
    st = _two_peer_state(NewPeerGaterParams(0.1, 0.9, 0.999))
    now = 10 * Second
    v = st.view()
    lib.orc_gater_event(v, 0, 0, 0, st.GATE_VALIDATE)
    lib.orc_gater_event(v, 0, 0, 0, st.GATE_THROTTLE)
    for _ in range(30):
        lib.orc_gater_event(v, 0, 0, 0, st.GATE_DUPLICATE)
    for _ in range(3):
        lib.orc_gater_event(v, 0, 0, 0, st.GATE_DELIVER)
    lib.orc_gater_round_end(v, now)
    lib.orc_gater_round_begin(v, now)
    n = 20000
    acc = sum(lib.orc_gater_accept(v, 7, g, 0, 0, 3) for g in range(n))
    p = (1 + 3) / (1 + 3 + 0.125 * 30)
    assert abs(acc / n - p) < 4 * np.sqrt(p * (1 - p) / n)
    assert st.gater_throttled() == n - acc


# ---- GPU -------------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("weights,shards", [(None, 0), ({0: 0.5, 2: 2.25}, 0), (None, 2), ({0: 0.5, 2: 2.25}, 3)])
def test_gater_network_bit_exact(require_gpu, weights, shards):
    """A network whose validations often throttle (so every router's gate
    turns on), sybils sharing IPs (shared stats), churn and gossip: the
    engine's gater state, its drops and everything the gated deliveries touch
    equal the oracle's after every tick.  On 2 / 3 shards too: each router's
    gate on its shard, pushed copies gated at the receiving shard."""
    from fixtures import beacon_params, sybil_ips, synthetic_state
    from gsim.engine import random_regular
    from gsim.params import GossipSubParams, PeerScoreThresholds
    from test_heartbeat import tick_time
    from tickrun import run_parity, subscribed_schedule
    n, k, T = 800, 16, 3
    rng = np.random.default_rng(404)
    net = random_regular(n, k, seed=77, n_topics=T)
    net.ip_ptr, net.ip_ids, net.n_ips = sybil_ips(n, 0.3, 6, rng)
    params = beacon_params(T)
    gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-100, GraylistThreshold=-400)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 6 / k)
    ticks = list(range(1, 7))
    sched = subscribed_schedule(rng, ticks, net, T, 12.0, 0.0, verdicts=(0.45, 0.15, 0.1, 0.25, 0.05))
    src = np.repeat(np.arange(n, dtype=np.uint32), np.diff(net.row_ptr.astype(np.int64)))
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=40, replace=False)]
    churn = {3: [(down, False)], 5: [(down, True)]}
    gater = NewPeerGaterParams(0.05, 0.9, 0.99)
    if weights:
        gater.TopicDeliveryWeights = weights
    log = []
    eng = None
    if shards:
        from gsim.shard import ShardedEngine
        from tickrun import SEED
        eng = ShardedEngine(params, th, gossip=gp, shards=shards)
        eng.load_graph(net)
        eng.set_seed(SEED)
        st.push_to_engine(eng)
    run_parity(net, params, th, gp, st, ticks, sched, ring=512, churn=churn, gater=gater, gater_log=log, eng=eng)
    assert log[-1] > 100, f"the gate should have dropped copies: {log}"


@pytest.mark.gpu
def test_gater_refuses_new_ips(require_gpu):
    """The gater's per-IP groups are built from the IPs at gsim_set_peer_gater
    (peer_gater.go getPeerIP at AddPeer): replacing the IPs afterwards is
    refused (GSIM_ESTATE) rather than leaving the groups stale."""
    from fixtures import beacon_params
    from gsim import _abi
    from gsim.engine import Engine, GsimError, random_regular
    n = 200
    net = random_regular(n, 8, seed=3, n_topics=1)
    ip_ptr = np.arange(n + 1, dtype=np.uint32)
    ip_ids = (np.arange(n) // 4).astype(np.uint32)
    from fixtures import beacon_thresholds
    eng = Engine(beacon_params(1), beacon_thresholds())
    try:
        eng.load_graph(net)
        eng.set_ips(ip_ptr, ip_ids, n // 4)                 # before the gater: fine
        eng.msgs_init(64, 10, 0, 10**9)
        eng.set_peer_gater(NewPeerGaterParams(0.05, 0.9, 0.99))
        with pytest.raises(GsimError) as ex:
            eng.set_ips(ip_ptr, np.arange(n, dtype=np.uint32), n)
        assert ex.value.rc == _abi.GSIM_ESTATE
    finally:
        eng.close()
