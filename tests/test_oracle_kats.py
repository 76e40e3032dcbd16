"""The reference's own known-answer tests, run against the CPU oracle.

Each test restates one Go test from score_test.go / mcache_test.go /
gossip_tracer_test.go / timecache/*_test.go with the same inputs and the same
expected literals.  Sleep-based reference tests run on a virtual clock, so
their `>=`/variance checks become exact equalities here (noted per test).
These pin the oracle before it is trusted as the GPU parity checker.
"""
import ipaddress
import math

import numpy as np
import pytest

import oracle_binding as ob
from gsim.params import Millisecond, PeerScoreParams, Second, TopicScoreParams
from peerscore_harness import Msg, PeerScore

R = {name: i for i, name in enumerate([
    "BLACKLISTED_PEER", "BLACKLISTED_SOURCE", "MISSING_SIGNATURE", "UNEXPECTED_SIGNATURE", "UNEXPECTED_AUTH_INFO",
    "INVALID_SIGNATURE", "VALIDATION_QUEUE_FULL", "VALIDATION_THROTTLED", "VALIDATION_FAILED",
    "VALIDATION_IGNORED", "SELF_ORIGIN"])}

MY = "mytopic"


def params_with(tp=None, **kw):
    p = PeerScoreParams(AppSpecificScore=lambda p: 0.0, **kw)
    if tp is not None:
        p.Topics[MY] = tp
    return p


# ---- score_test.go -----------------------------------------------------------

def test_score_time_in_mesh():
    """score_test.go:13-50 (reference asserts >=; exact on the virtual clock)."""
    tp = TopicScoreParams(TopicWeight=0.5, TimeInMeshWeight=1, TimeInMeshQuantum=Millisecond, TimeInMeshCap=3600)
    ps = PeerScore(params_with(tp), peers=["A"])
    ps.AddPeer("A")
    assert ps.Score("A") == 0
    ps.Graft("A", MY)
    elapsed = tp.TimeInMeshQuantum * 200
    ps.sleep(elapsed)
    ps.refreshScores()
    expected = tp.TopicWeight * tp.TimeInMeshWeight * float(elapsed // tp.TimeInMeshQuantum)
    assert ps.Score("A") == expected == 100.0


def test_score_time_in_mesh_cap():
    """score_test.go:52-84 (reference: within 50% variance; exact here)."""
    tp = TopicScoreParams(TopicWeight=0.5, TimeInMeshWeight=1, TimeInMeshQuantum=Millisecond, TimeInMeshCap=10)
    ps = PeerScore(params_with(tp), peers=["A"])
    ps.AddPeer("A")
    ps.Graft("A", MY)
    ps.sleep(tp.TimeInMeshQuantum * 40)
    ps.refreshScores()
    assert ps.Score("A") == tp.TopicWeight * tp.TimeInMeshWeight * tp.TimeInMeshCap == 5.0


def _deliver_first(ps, n, frm="A"):
    for i in range(n):
        m = Msg(i, MY, frm)
        ps.ValidateMessage(m)
        ps.DeliverMessage(m)


def test_score_first_message_deliveries():
    """score_test.go:86-124: 100 first deliveries -> 100."""
    tp = TopicScoreParams(TopicWeight=1, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=1.0,
                          FirstMessageDeliveriesCap=2000, TimeInMeshQuantum=Second)
    ps = PeerScore(params_with(tp), peers=["A"])
    ps.AddPeer("A")
    ps.Graft("A", MY)
    _deliver_first(ps, 100)
    ps.refreshScores()
    assert ps.Score("A") == 100.0


def test_score_first_message_deliveries_cap():
    """score_test.go:126-164: capped at 50."""
    tp = TopicScoreParams(TopicWeight=1, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=1.0,
                          FirstMessageDeliveriesCap=50, TimeInMeshQuantum=Second)
    ps = PeerScore(params_with(tp), peers=["A"])
    ps.AddPeer("A")
    ps.Graft("A", MY)
    _deliver_first(ps, 100)
    ps.refreshScores()
    assert ps.Score("A") == 50.0


def test_score_first_message_deliveries_decay():
    """score_test.go:166-215: 90 then x0.9 per refresh, by repeated multiplication."""
    tp = TopicScoreParams(TopicWeight=1, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=0.9,
                          FirstMessageDeliveriesCap=2000, TimeInMeshQuantum=Second)
    ps = PeerScore(params_with(tp), peers=["A"])
    ps.AddPeer("A")
    ps.Graft("A", MY)
    _deliver_first(ps, 100)
    ps.refreshScores()
    expected = tp.TopicWeight * tp.FirstMessageDeliveriesWeight * tp.FirstMessageDeliveriesDecay * 100.0
    assert ps.Score("A") == expected
    for _ in range(10):
        ps.refreshScores()
        expected *= tp.FirstMessageDeliveriesDecay
    assert ps.Score("A") == expected


def test_score_mesh_message_deliveries():
    """score_test.go:217-308: A first, B within the 10ms window, C after it."""
    tp = TopicScoreParams(TopicWeight=1, MeshMessageDeliveriesWeight=-1,
                          MeshMessageDeliveriesActivation=Second, MeshMessageDeliveriesWindow=10 * Millisecond,
                          MeshMessageDeliveriesThreshold=20, MeshMessageDeliveriesCap=100,
                          MeshMessageDeliveriesDecay=1.0, FirstMessageDeliveriesWeight=0, TimeInMeshQuantum=Second)
    ps = PeerScore(params_with(tp), peers=["A", "B", "C"])
    for p in "ABC":
        ps.AddPeer(p)
        ps.Graft(p, MY)
    ps.refreshScores()
    for p in "ABC":
        assert ps.Score(p) >= 0
    ps.sleep(tp.MeshMessageDeliveriesActivation)
    late = []
    for i in range(100):
        m = Msg(i, MY, "A")
        ps.ValidateMessage(m)
        ps.DeliverMessage(m)
        ps.DuplicateMessage(Msg(i, MY, "B"))
        late.append(Msg(i, MY, "C"))
    ps.sleep(tp.MeshMessageDeliveriesWindow + 20 * Millisecond)   # time.AfterFunc(window+20ms)
    for m in late:
        ps.DuplicateMessage(m)
    # refresh at t0+1.03s: meshTime 1.03s > activation 1s -> active
    ps.refreshScores()
    assert ps.Score("A") >= 0
    assert ps.Score("B") >= 0
    penalty = tp.MeshMessageDeliveriesThreshold * tp.MeshMessageDeliveriesThreshold
    assert ps.Score("C") == tp.TopicWeight * tp.MeshMessageDeliveriesWeight * penalty == -400.0


def test_score_mesh_message_deliveries_decay():
    """score_test.go:310-369: -(20 - 40*0.9^21)^2 = -244.08564168167945 (re-derived in fp64)."""
    tp = TopicScoreParams(TopicWeight=1, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesActivation=0,
                          MeshMessageDeliveriesWindow=10 * Millisecond, MeshMessageDeliveriesThreshold=20,
                          MeshMessageDeliveriesCap=100, MeshMessageDeliveriesDecay=0.9,
                          FirstMessageDeliveriesWeight=0, TimeInMeshQuantum=Second)
    ps = PeerScore(params_with(tp), peers=["A"])
    ps.AddPeer("A")
    ps.Graft("A", MY)
    _deliver_first(ps, 40)
    ps.sleep(1)   # activation is meshTime > 0 (strict): the reference's test takes real time here
    ps.refreshScores()
    assert ps.Score("A") >= 0
    decayed = 40.0 * tp.MeshMessageDeliveriesDecay
    for _ in range(20):
        ps.refreshScores()
        decayed *= tp.MeshMessageDeliveriesDecay
    deficit = tp.MeshMessageDeliveriesThreshold - decayed
    expected = tp.TopicWeight * tp.MeshMessageDeliveriesWeight * (deficit * deficit)
    got = ps.Score("A")
    assert got == expected
    assert got == -244.08564168167945


def test_score_mesh_failure_penalty():
    """score_test.go:371-450: prune of an under-delivering peer -> -400."""
    tp = TopicScoreParams(TopicWeight=1, MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=1.0,
                          MeshMessageDeliveriesActivation=0, MeshMessageDeliveriesWindow=10 * Millisecond,
                          MeshMessageDeliveriesThreshold=20, MeshMessageDeliveriesCap=100,
                          MeshMessageDeliveriesDecay=1.0, MeshMessageDeliveriesWeight=0,
                          FirstMessageDeliveriesWeight=0, TimeInMeshQuantum=Second)
    ps = PeerScore(params_with(tp), peers=["A", "B"])
    for p in "AB":
        ps.AddPeer(p)
        ps.Graft(p, MY)
    _deliver_first(ps, 100)
    ps.sleep(1)
    ps.refreshScores()
    assert ps.Score("A") == 0 and ps.Score("B") == 0
    ps.Prune("B", MY)
    ps.refreshScores()
    assert ps.Score("A") == 0
    assert ps.Score("B") == -400.0


def _reject_n(ps, n, reason, validate=False):
    for i in range(n):
        m = Msg(i, MY, "A")
        if validate:
            ps.ValidateMessage(m)
        ps.RejectMessage(m, reason)


def test_score_invalid_message_deliveries():
    """score_test.go:452-487: -10000."""
    tp = TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second, InvalidMessageDeliveriesWeight=-1,
                          InvalidMessageDeliveriesDecay=1.0)
    ps = PeerScore(params_with(tp), peers=["A"])
    ps.AddPeer("A")
    ps.Graft("A", MY)
    _reject_n(ps, 100, R["INVALID_SIGNATURE"])
    ps.refreshScores()
    assert ps.Score("A") == -10000.0


def test_score_invalid_message_deliveries_decay():
    """score_test.go:489-534: -(0.9*100)^2 then x0.81 per refresh; -984.770902183612 after 10."""
    tp = TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second, InvalidMessageDeliveriesWeight=-1,
                          InvalidMessageDeliveriesDecay=0.9)
    ps = PeerScore(params_with(tp), peers=["A"])
    ps.AddPeer("A")
    ps.Graft("A", MY)
    _reject_n(ps, 100, R["INVALID_SIGNATURE"])
    ps.refreshScores()
    expected = tp.TopicWeight * tp.InvalidMessageDeliveriesWeight * math.pow(tp.InvalidMessageDeliveriesDecay * 100, 2)
    assert ps.Score("A") == expected
    for _ in range(10):
        ps.refreshScores()
        expected *= math.pow(tp.InvalidMessageDeliveriesDecay, 2)
    # the reference compares against repeated x0.81 while the counter decays by x0.9: equal in fp64
    assert ps.Score("A") == expected
    assert ps.Score("A") == pytest.approx(-984.770902183612, rel=1e-15)


def test_score_reject_message_deliveries():
    """score_test.go:536-666: ignore/throttle have no effect; failures give -1 then -4."""
    tp = TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second, InvalidMessageDeliveriesWeight=-1,
                          InvalidMessageDeliveriesDecay=1.0)
    ps = PeerScore(params_with(tp), peers=["A", "B"])
    ps.AddPeer("A")
    ps.AddPeer("B")
    msg = Msg(0, MY, "A")
    msg2 = Msg(0, MY, "B")
    ps.RejectMessage(msg, R["BLACKLISTED_PEER"])
    ps.RejectMessage(msg, R["BLACKLISTED_SOURCE"])
    ps.RejectMessage(msg, R["VALIDATION_QUEUE_FULL"])
    assert ps.Score("A") == 0.0
    ps.ValidateMessage(msg)
    ps.RejectMessage(msg, R["VALIDATION_THROTTLED"])
    ps.DuplicateMessage(msg2)
    assert ps.Score("A") == 0.0 and ps.Score("B") == 0.0
    ps.expire_head_now()
    ps.gc_deliveries()
    ps.ValidateMessage(msg)
    ps.RejectMessage(msg, R["VALIDATION_IGNORED"])
    ps.DuplicateMessage(msg2)
    assert ps.Score("A") == 0.0 and ps.Score("B") == 0.0
    ps.expire_head_now()
    ps.gc_deliveries()
    ps.ValidateMessage(msg)
    ps.RejectMessage(msg, R["VALIDATION_FAILED"])
    ps.DuplicateMessage(msg2)
    assert ps.Score("A") == -1.0 and ps.Score("B") == -1.0
    ps.expire_head_now()
    ps.gc_deliveries()
    ps.ValidateMessage(msg)
    ps.DuplicateMessage(msg2)
    ps.RejectMessage(msg, R["VALIDATION_FAILED"])
    assert ps.Score("A") == -4.0 and ps.Score("B") == -4.0


def test_score_application_score():
    """score_test.go:668-694: P5 * 0.5 for i in [-100, 100)."""
    val = {"v": 0.0}
    params = PeerScoreParams(AppSpecificScore=lambda p: val["v"], AppSpecificWeight=0.5)
    ps = PeerScore(params, peers=["A"], extra_topics=[MY])
    ps.AddPeer("A")
    ps.Graft("A", MY)   # unscored topic: no stats created (score.go:888-891)
    for i in range(-100, 100):
        val["v"] = float(i)
        ps.refreshScores()
        assert ps.Score("A") == float(i) * params.AppSpecificWeight


IPS = {"A": ["1.2.3.4"], "B": ["2.3.4.5"], "C": ["2.3.4.5", "3.4.5.6"], "D": ["2.3.4.5"]}


def test_score_ip_colocation():
    """score_test.go:696-744: three peers share 2.3.4.5 -> -(3-1)^2 = -4 each."""
    params = PeerScoreParams(AppSpecificScore=lambda p: 0.0, IPColocationFactorThreshold=1,
                             IPColocationFactorWeight=-1)
    ps = PeerScore(params, peers=list("ABCD"), extra_topics=[MY], ips=IPS)
    for p in "ABCD":
        ps.AddPeer(p)
        ps.Graft(p, MY)
    ps.refreshScores()
    assert ps.Score("A") == 0
    for p in "BCD":
        assert ps.Score(p) == params.IPColocationFactorWeight * float((3 - 1) ** 2) == -4.0


def test_score_ip_colocation_whitelist():
    """score_test.go:746-803: 2.3.0.0/16 whitelisted -> all zero."""
    params = PeerScoreParams(AppSpecificScore=lambda p: 0.0, IPColocationFactorThreshold=1,
                             IPColocationFactorWeight=-1,
                             IPColocationFactorWhitelist=[ipaddress.ip_network("2.3.0.0/16")])
    ps = PeerScore(params, peers=list("ABCD"), extra_topics=[MY], ips=IPS)
    for p in "ABCD":
        ps.AddPeer(p)
        ps.Graft(p, MY)
    ps.refreshScores()
    for p in "ABCD":
        assert ps.Score(p) == 0


def test_score_behaviour_penalty():
    """score_test.go:805-859: -1, -4, then -3.9204 after one decay at 0.99."""
    params = PeerScoreParams(AppSpecificScore=lambda p: 0.0, BehaviourPenaltyWeight=-1, BehaviourPenaltyDecay=0.99)
    ps = PeerScore(params, peers=["A"])
    ps.AddPenalty("A", 1)                 # non-existent peer: no-op
    assert ps.Score("A") == 0
    ps.AddPeer("A")
    assert ps.Score("A") == 0
    ps.AddPenalty("A", 1)
    assert ps.Score("A") == -1
    ps.AddPenalty("A", 1)
    assert ps.Score("A") == -4
    ps.refreshScores()
    assert ps.Score("A") == -3.9204


def test_score_retention():
    """score_test.go:861-903 (virtual clock: exact at RetainScore/2 and after expiry)."""
    params = PeerScoreParams(AppSpecificScore=lambda p: -1000.0, AppSpecificWeight=1.0, RetainScore=Second)
    ps = PeerScore(params, peers=["A"], extra_topics=[MY])
    ps.AddPeer("A")
    ps.Graft("A", MY)
    ps.refreshScores()
    assert ps.Score("A") == -1000.0
    ps.RemovePeer("A")
    delay = params.RetainScore // 2
    ps.sleep(delay)
    ps.refreshScores()
    assert ps.Score("A") == -1000.0
    ps.sleep(delay + 50 * Millisecond)
    ps.refreshScores()
    assert ps.Score("A") == 0


def test_score_recap_topic_params():
    """score_test.go:905-1000: caps 100 -> 50 recap first (A) and mesh (B) counters."""
    def tp(cap):
        return TopicScoreParams(TopicWeight=1, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesActivation=Second,
                                MeshMessageDeliveriesWindow=10 * Millisecond, MeshMessageDeliveriesThreshold=20,
                                MeshMessageDeliveriesCap=cap, MeshMessageDeliveriesDecay=1.0,
                                FirstMessageDeliveriesWeight=10, FirstMessageDeliveriesDecay=1.0,
                                FirstMessageDeliveriesCap=cap, TimeInMeshQuantum=Second)
    ps = PeerScore(params_with(tp(100)), peers=["A", "B"])
    for p in "AB":
        ps.AddPeer(p)
        ps.Graft(p, MY)
    for i in range(100):
        m = Msg(i, MY, "A")
        ps.ValidateMessage(m)
        ps.DeliverMessage(m)
        ps.DuplicateMessage(Msg(i, MY, "B"))
    assert ps.topic_stat("A", MY, "first") == 100
    assert ps.topic_stat("B", MY, "meshd") == 100
    ps.SetTopicScoreParams(MY, tp(50))
    assert ps.topic_stat("A", MY, "first") == 50
    assert ps.topic_stat("B", MY, "meshd") == 50


def test_score_reset_topic_params():
    """score_test.go:1002-1062: -10000 then -100000 after the weight changes."""
    ps = PeerScore(params_with(TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second,
                                                InvalidMessageDeliveriesWeight=-1,
                                                InvalidMessageDeliveriesDecay=1.0)), peers=["A"])
    ps.AddPeer("A")
    _reject_n(ps, 100, R["VALIDATION_FAILED"], validate=True)
    assert ps.Score("A") == -10000
    ps.SetTopicScoreParams(MY, TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second,
                                                InvalidMessageDeliveriesWeight=-10,
                                                InvalidMessageDeliveriesDecay=1.0))
    assert ps.Score("A") == -100000


# ---- mcache_test.go ------------------------------------------------------------

def test_message_cache():
    """mcache_test.go:11-154: exact gossip-id order across shifts."""
    lib = ob.load()
    mc = lib.orc_mcache_new(3, 5)
    T = 0

    def gids():
        out = np.zeros(100, dtype=np.uint64)
        n = lib.orc_mcache_gossip_ids(mc, T, out.ctypes.data, 100)
        return list(out[:n])

    for i in range(10):
        lib.orc_mcache_put(mc, i, T)
    for i in range(10):
        assert lib.orc_mcache_get(mc, i)
    g = gids()
    assert g == list(range(10))
    lib.orc_mcache_shift(mc)
    for i in range(10, 20):
        lib.orc_mcache_put(mc, i, T)
    for i in range(20):
        assert lib.orc_mcache_get(mc, i)
    g = gids()
    assert len(g) == 20
    assert g[10:] == list(range(10)) and g[:10] == list(range(10, 20))
    for lo in (20, 30, 40, 50):
        lib.orc_mcache_shift(mc)
        for i in range(lo, lo + 10):
            lib.orc_mcache_put(mc, i, T)
    assert lib.orc_mcache_len(mc) == 50
    for i in range(10):
        assert not lib.orc_mcache_get(mc, i)
    for i in range(10, 60):
        assert lib.orc_mcache_get(mc, i)
    g = gids()
    assert len(g) == 30
    assert g[:10] == list(range(50, 60))
    assert g[10:20] == list(range(40, 50))
    assert g[20:30] == list(range(30, 40))
    lib.orc_mcache_free(mc)


def test_message_cache_get_for_peer_counts_and_shift_reset():
    """mcache.go:66-80 retransmission counter; Shift drops peertx (mcache.go:94-104)."""
    lib = ob.load()
    mc = lib.orc_mcache_new(3, 5)
    import ctypes
    lib.orc_mcache_put(mc, 7, 0)
    cnt = ctypes.c_int32()
    for k in range(1, 5):
        assert lib.orc_mcache_get_for_peer(mc, 7, 1, ctypes.byref(cnt)) == 1
        assert cnt.value == k
    assert lib.orc_mcache_get_for_peer(mc, 7, 2, ctypes.byref(cnt)) == 1 and cnt.value == 1
    for _ in range(5):
        lib.orc_mcache_shift(mc)
    assert lib.orc_mcache_get_for_peer(mc, 7, 1, ctypes.byref(cnt)) == 0
    lib.orc_mcache_free(mc)


def test_new_message_cache_rejects_gossip_gt_history():
    """mcache.go:21-26 panics; the oracle returns NULL."""
    assert ob.load().orc_mcache_new(6, 5) is None


# ---- gossip_tracer_test.go -----------------------------------------------------

def test_broken_promises():
    """gossip_tracer_test.go:12-64."""
    lib = ob.load()
    follow = 100 * Millisecond
    gt = lib.orc_gtracer_new(follow)
    mids = np.arange(100, dtype=np.uint64)
    now = 0
    for peer in (1, 2, 3):   # A, B, C
        lib.orc_gtracer_add_promise(gt, peer, mids.ctypes.data, 100, 17, now)
    peers = np.zeros(8, dtype=np.uint32)
    counts = np.zeros(8, dtype=np.int32)
    assert lib.orc_gtracer_broken(gt, now, peers.ctypes.data, counts.ctypes.data, 8) == 0
    lib.orc_gtracer_throttle(gt, 3)
    now += follow + Millisecond
    n = lib.orc_gtracer_broken(gt, now, peers.ctypes.data, counts.ctypes.data, 8)
    assert n == 2
    assert list(peers[:2]) == [1, 2] and list(counts[:2]) == [1, 1]
    assert lib.orc_gtracer_peer_promises(gt) == 0
    lib.orc_gtracer_free(gt)


def test_no_broken_promises():
    """gossip_tracer_test.go:66-103."""
    lib = ob.load()
    follow = 100 * Millisecond
    gt = lib.orc_gtracer_new(follow)
    mids = np.arange(100, dtype=np.uint64)
    lib.orc_gtracer_add_promise(gt, 1, mids.ctypes.data, 100, 5, 0)
    lib.orc_gtracer_add_promise(gt, 2, mids.ctypes.data, 100, 93, 0)
    for m in range(100):
        lib.orc_gtracer_fulfill(gt, m)
    peers = np.zeros(8, dtype=np.uint32)
    counts = np.zeros(8, dtype=np.int32)
    assert lib.orc_gtracer_broken(gt, follow + Millisecond, peers.ctypes.data, counts.ctypes.data, 8) == 0
    assert lib.orc_gtracer_peer_promises(gt) == 0
    lib.orc_gtracer_free(gt)


# ---- timecache/*_test.go ---------------------------------------------------------

@pytest.mark.parametrize("strategy", [0, 1])
def test_timecache_found(strategy):
    """first_seen_cache_test.go:9-17, last_seen_cache_test.go:9-17."""
    lib = ob.load()
    c = lib.orc_tcache_new(strategy, 60 * Second)
    lib.orc_tcache_add(c, 42, 0)
    assert lib.orc_tcache_has(c, 42, 0)
    lib.orc_tcache_free(c)


@pytest.mark.parametrize("strategy,n", [(0, 10), (1, 11)])
def test_timecache_expire(strategy, n):
    """first_seen_cache_test.go:19-35 / last_seen_cache_test.go:19-34 (1s sweep, 1s TTL)."""
    lib = ob.load()
    c = lib.orc_tcache_new(strategy, Second)
    now = 0
    for i in range(n):
        lib.orc_tcache_add(c, i, now)
        now += 100 * Millisecond
    now += 2 * Second
    lib.orc_tcache_sweep(c, now - Second)     # the 1 s ticker fired at least once after expiry
    lib.orc_tcache_sweep(c, now)
    for i in range(n):
        assert not lib.orc_tcache_has(c, i, now)
    lib.orc_tcache_free(c)


def test_last_seen_cache_slide_forward():
    """last_seen_cache_test.go:36-86 (skipped in the reference's CI; exact on a virtual clock)."""
    lib = ob.load()
    c = lib.orc_tcache_new(1, Second)
    now = 0
    for i in range(8):
        lib.orc_tcache_add(c, i, now)
        now += 100 * Millisecond
    assert lib.orc_tcache_has(c, 0, now)          # T800: slides 0 to 1800
    now += 400 * Millisecond
    lib.orc_tcache_sweep(c, now)                  # T1200
    assert lib.orc_tcache_has(c, 0, now)          # slides to 2200
    assert not lib.orc_tcache_has(c, 1, now)
    now += 1100 * Millisecond
    lib.orc_tcache_sweep(c, now)                  # T2300
    assert not lib.orc_tcache_has(c, 0, now)
    assert not lib.orc_tcache_has(c, 0, now)
    lib.orc_tcache_free(c)


def test_first_seen_does_not_slide():
    """first_seen_cache.go:47-56: Add of an existing id keeps the original expiry."""
    lib = ob.load()
    c = lib.orc_tcache_new(0, Second)
    assert lib.orc_tcache_add(c, 1, 0) == 1
    assert lib.orc_tcache_add(c, 1, 900 * Millisecond) == 0
    lib.orc_tcache_sweep(c, 1001 * Millisecond)
    assert not lib.orc_tcache_has(c, 1, 1001 * Millisecond)
    lib.orc_tcache_free(c)


# ---- Philox4x32-10 known-answer vectors (Random123 kat_vectors) ----------------

@pytest.mark.parametrize("ctr,key,out", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_kat(ctr, key, out):
    lib = ob.load()
    c = np.array(ctr, dtype=np.uint32)
    k = np.array(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib.orc_philox4x32_10(c.ctypes.data, k.ctypes.data, o.ctypes.data)
    assert tuple(int(x) for x in o) == out
