"""GPU parity: fused refreshScores+score and ipColocationFactor kernels vs the
CPU oracle, bit-exact (both compiled with -ffp-contract=off), plus the
reference's own scoring KATs replayed through the engine via state writes."""
import numpy as np
import pytest

import oracle_binding as ob
from fixtures import beacon_params, beacon_thresholds, randomize_state, sybil_ips
from gsim import _abi
from gsim.engine import Engine, random_regular
from gsim.params import Millisecond, PeerScoreParams, PeerScoreThresholds, Second, TopicScoreParams

pytestmark = pytest.mark.gpu

NOW = 5_000 * Second


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64) if a.dtype.itemsize == 8 else a


def assert_state_equal(st_cpu, st_gpu, fields):
    for f in fields:
        a, b = getattr(st_cpu, f), getattr(st_gpu, f)
        if not np.array_equal(bits(a), bits(b)):
            bad = np.argwhere(bits(a) != bits(b))
            idx = tuple(bad[0])
            raise AssertionError(f"{f}: {len(bad)} mismatches, first at {idx}: cpu={a[idx]!r} gpu={b[idx]!r}")


def multi_ips(n, rng, pool):
    """0-3 IPs per peer drawn from a small shared pool: peers with no IP, one IP
    and several IPs (ipColocationFactor counts a peer once per IP it shares)."""
    cnt = rng.choice([0, 1, 1, 1, 2, 3], size=n)
    ip_ptr = np.zeros(n + 1, dtype=np.uint32)
    ip_ptr[1:] = np.cumsum(cnt)
    ids = [np.sort(rng.choice(pool, size=c, replace=False)) for c in cnt]
    ip_ids = np.concatenate(ids).astype(np.uint32) if ip_ptr[-1] else np.zeros(0, np.uint32)
    return ip_ptr, ip_ids, pool


def build(n, k, T, seed, frac_sybil=0.2, topic_cap=0.0, multi_ip=False, hub_cap=0):
    rng = np.random.default_rng(seed)
    if hub_cap:
        # power law with hub rows above 64 connections (k_ip_colocation_hub) up to hub_cap
        from gsim import graphs
        net = graphs.power_law(n, k, 2.1, hub_cap, seed=seed, n_topics=T, i0=1.0)
        assert int(np.diff(net.row_ptr.astype(np.int64)).max()) > 256
    else:
        net = random_regular(n, k, seed=seed, n_topics=T)
    if multi_ip:
        net.ip_ptr, net.ip_ids, net.n_ips = multi_ips(n, rng, pool=max(8, n // 40))
    else:
        net.ip_ptr, net.ip_ids, net.n_ips = sybil_ips(n, frac_sybil, 5, rng)
    params = beacon_params(T, topic_cap=topic_cap)
    p5 = np.where(rng.random(n) < 0.1, -1000.0 * rng.random(n), rng.normal(0, 5, n))
    white = (rng.random(net.n_ips) < 0.1).astype(np.uint8)
    st = ob.NetState(net, params, thresholds=beacon_thresholds(), p5=p5, ip_white=white)
    randomize_state(st, rng, NOW)
    return net, params, st, p5, white


@pytest.mark.parametrize("n,k,T,cap,multi_ip,hub_cap", [(600, 16, 1, 0.0, False, 0), (2000, 32, 4, 0.0, False, 0),
                                                        (3000, 32, 3, 3.5, False, 0), (1000, 20, 11, 0.0, False, 0),
                                                        (1500, 24, 2, 0.0, True, 0), (6000, 12, 2, 0.0, False, 2000),
                                                        (6000, 12, 2, 0.0, True, 2000)])
def test_refresh_and_score_bit_exact(require_gpu, n, k, T, cap, multi_ip, hub_cap):
    """hub_cap: a power law whose hub rows (65-2000 connections) take the
    sorted-key P6 path (k_ip_colocation_hub), sybil IPs shared by dozens of a
    hub's members, or several IPs per peer (the hub's per-IP scan)."""
    net, params, st, p5, white = build(n, k, T, seed=n + T, topic_cap=cap, multi_ip=multi_ip, hub_cap=hub_cap,
                                       frac_sybil=0.4 if hub_cap else 0.2)
    eng = Engine(params, beacon_thresholds())
    eng.load_graph(net)
    eng.set_app_score(p5)
    eng.set_ip_whitelist(white)
    st.push_to_engine(eng)
    lib = ob.load()
    v = st.view()
    for step in range(3):
        now = NOW + step * Second
        eng.refresh_scores(now)
        lib.orc_refresh_scores(v, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
        gpu = ob.NetState(net, params, thresholds=beacon_thresholds(), p5=p5, ip_white=white)
        gpu.pull_from_engine(eng)
        assert_state_equal(st, gpu, ["first", "meshd", "fail", "invalid", "mesh_time", "tflags", "bp", "estate",
                                     "expire", "p6", "score"])
        assert np.array_equal(bits(eng.scores()), bits(st.score))
    eng.close()


def test_compute_scores_without_decay(require_gpu):
    net, params, st, p5, white = build(1500, 24, 2, seed=7)
    eng = Engine(params, beacon_thresholds())
    eng.load_graph(net)
    eng.set_app_score(p5)
    eng.set_ip_whitelist(white)
    st.push_to_engine(eng)
    eng.compute_scores()
    lib = ob.load()
    v = st.view()
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    assert np.array_equal(bits(eng.scores()), bits(st.score))
    eng.close()


def test_set_topic_params_recap_matches_oracle(require_gpu):
    net, params, st, p5, white = build(800, 16, 2, seed=11)
    eng = Engine(params, beacon_thresholds())
    eng.load_graph(net)
    st.push_to_engine(eng)
    name = eng.topics[1]
    newp = beacon_topic_lower(params.Topics[name])
    eng.set_topic_score_params(name, newp)
    c = newp.to_c(True)
    import ctypes
    lib = ob.load()
    slot = ctypes.cast(ctypes.addressof(st.tp) + 1 * ctypes.sizeof(_abi.CTopicScoreParams), ctypes.c_void_p)
    lib.orc_set_topic_params(st.view(), 1, slot, ctypes.cast(ctypes.byref(c), ctypes.c_void_p))
    gpu = ob.NetState(net, params)
    gpu.pull_from_engine(eng)
    assert_state_equal(st, gpu, ["first", "meshd"])
    eng.close()


def beacon_topic_lower(tp):
    from dataclasses import replace
    return replace(tp, FirstMessageDeliveriesCap=7.5, MeshMessageDeliveriesCap=33.0)


# ---- score_test.go KATs replayed on the GPU (state set through the ABI) ---------

def _single(params, topics=("mytopic",), ips=None):
    from peerscore_harness import star_network
    net, names = star_network(["A", "B", "C", "D"], len(topics), ips)
    eng = Engine(params, PeerScoreThresholds(), topics=list(topics), validate=False)
    eng.load_graph(net)
    return eng, net, names


def test_gpu_kat_behaviour_penalty(require_gpu):
    """score_test.go:805-859: -1, -4, -3.9204."""
    eng, net, _ = _single(PeerScoreParams(AppSpecificScore=lambda p: 0.0, BehaviourPenaltyWeight=-1,
                                          BehaviourPenaltyDecay=0.99))
    bp = np.zeros(net.e)
    for v, want in [(1.0, -1.0), (2.0, -4.0)]:
        bp[0] = v
        eng.write(_abi.F_BP, bp)
        eng.compute_scores()
        assert eng.scores()[0] == want
    eng.refresh_scores(1)
    assert eng.scores()[0] == -3.9204
    eng.close()


def test_gpu_kat_mesh_delivery_decay(require_gpu):
    """score_test.go:310-369: -244.08564168167945."""
    tp = TopicScoreParams(TopicWeight=1, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesActivation=0,
                          MeshMessageDeliveriesWindow=10 * Millisecond, MeshMessageDeliveriesThreshold=20,
                          MeshMessageDeliveriesCap=100, MeshMessageDeliveriesDecay=0.9,
                          FirstMessageDeliveriesWeight=0, TimeInMeshQuantum=Second)
    eng, net, _ = _single(PeerScoreParams(AppSpecificScore=lambda p: 0.0, Topics={"mytopic": tp}))
    meshd = np.zeros((1, net.e))
    meshd[0, 0] = 40
    tfl = np.zeros((1, net.e), dtype=np.uint8)
    tfl[0, 0] = _abi.TF_IN_MESH
    eng.write(_abi.F_MESHD, meshd)
    eng.write(_abi.F_TFLAGS, tfl)
    for i in range(21):
        eng.refresh_scores(1 + i)   # graftTime 0 -> meshTime > 0 activates
    assert eng.scores()[0] == -244.08564168167945
    eng.close()


def test_gpu_kat_ip_colocation_and_whitelist(require_gpu):
    """score_test.go:696-803: -4 for the three peers sharing 2.3.4.5; whitelist -> 0."""
    ips = {"A": ["1.2.3.4"], "B": ["2.3.4.5"], "C": ["2.3.4.5", "3.4.5.6"], "D": ["2.3.4.5"]}
    params = PeerScoreParams(AppSpecificScore=lambda p: 0.0, IPColocationFactorThreshold=1,
                             IPColocationFactorWeight=-1)
    eng, net, names = _single(params, ips=ips)
    eng.compute_scores()
    s = eng.scores()
    assert list(s[:4]) == [0.0, -4.0, -4.0, -4.0]
    import ipaddress
    params.IPColocationFactorWhitelist = [ipaddress.ip_network("2.3.0.0/16")]
    eng.set_ip_whitelist(np.array([params.whitelisted(ip) for ip in names], dtype=np.uint8))
    eng.compute_scores()
    assert list(eng.scores()[:4]) == [0.0, 0.0, 0.0, 0.0]
    eng.close()


def test_gpu_kat_retention(require_gpu):
    """score_test.go:861-903: retained -1000 until RetainScore elapses, then 0."""
    params = PeerScoreParams(AppSpecificScore=lambda p: -1000.0, AppSpecificWeight=1.0, RetainScore=Second)
    eng, net, _ = _single(params)
    eng.set_app_score(np.full(net.n, -1000.0))
    eng.refresh_scores(0)
    assert eng.scores()[0] == -1000.0
    est = eng.read(_abi.F_ESTATE)
    est[0] = _abi.ES_TRACKED
    exp = np.zeros(net.e, dtype=np.int64)
    exp[0] = params.RetainScore
    eng.write(_abi.F_ESTATE, est)
    eng.write(_abi.F_EXPIRE, exp)
    eng.refresh_scores(params.RetainScore // 2)
    assert eng.scores()[0] == -1000.0
    eng.refresh_scores(params.RetainScore + 50 * Millisecond)
    assert eng.scores()[0] == 0.0
    eng.close()


def test_gpu_kat_reset_topic_params(require_gpu):
    """score_test.go:1002-1062: -10000 -> -100000 after InvalidMessageDeliveriesWeight -1 -> -10."""
    tp = TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second, InvalidMessageDeliveriesWeight=-1,
                          InvalidMessageDeliveriesDecay=1.0)
    eng, net, _ = _single(PeerScoreParams(AppSpecificScore=lambda p: 0.0, Topics={"mytopic": tp}))
    inv = np.zeros((1, net.e))
    inv[0, 0] = 100
    eng.write(_abi.F_INVALID, inv)
    eng.compute_scores()
    assert eng.scores()[0] == -10000
    eng.set_topic_score_params("mytopic", TopicScoreParams(TopicWeight=1, TimeInMeshQuantum=Second,
                                                           InvalidMessageDeliveriesWeight=-10,
                                                           InvalidMessageDeliveriesDecay=1.0))
    eng.compute_scores()
    assert eng.scores()[0] == -100000
    eng.close()


@pytest.mark.parametrize("multi_ip", [False, True])
def test_ip_colocation_rows_over_4096_bit_exact(require_gpu, multi_ip):
    """A row of 6001 connections (peer 0 connected to every other peer, the
    leaves also on a random 8-regular graph): ipColocationFactor has no
    degree bound (score.go:344-388).  P6's hub kernel counts a row longer
    than its 4096-key LDS tile in tiles (members in chunks, every key tile
    sorted in turn); with several IPs per peer it scans per IP from memory.
    Sybil IPs shared by 10 peers, random tracked sets and whitelists; P6 and
    the scores equal the oracle's over three refreshes."""
    from gsim.engine import Network
    from gsim.graphs import _csr_from_pairs
    rng = np.random.default_rng(4097)
    n = 6002
    leaves = np.arange(1, n, dtype=np.int64)
    ring = rng.permutation(leaves)
    u = [np.zeros(n - 1, np.int64)]
    v = [leaves]
    for s_ in range(1, 5):                          # 4 shifts of a random cycle: 8-regular among the leaves
        u.append(ring)
        v.append(np.roll(ring, s_))
    u, v = np.concatenate(u), np.concatenate(v)
    row_ptr, col, outbound = _csr_from_pairs(n, u, v)
    assert int(np.diff(row_ptr.astype(np.int64)).max()) == n - 1
    T = 2
    sub = np.full(n, (1 << T) - 1, dtype=np.uint64)
    if multi_ip:
        ip_ptr, ip_ids, n_ips = multi_ips(n, rng, pool=n // 40)
    else:
        ip_ids = (np.arange(n) // 10).astype(np.uint32)
        ip_ptr, n_ips = np.arange(n + 1, dtype=np.uint32), int(ip_ids.max()) + 1
    net = Network(n, row_ptr, col, outbound, sub, ip_ptr, ip_ids, n_ips)
    params = beacon_params(T)
    p5 = rng.normal(0, 5, n)
    white = (rng.random(n_ips) < 0.1).astype(np.uint8)
    st = ob.NetState(net, params, thresholds=beacon_thresholds(), p5=p5, ip_white=white)
    randomize_state(st, rng, NOW)
    eng = Engine(params, beacon_thresholds())
    eng.load_graph(net)
    eng.set_app_score(p5)
    eng.set_ip_whitelist(white)
    st.push_to_engine(eng)
    lib = ob.load()
    v_ = st.view()
    for step in range(3):
        now = NOW + step * Second
        eng.refresh_scores(now)
        lib.orc_refresh_scores(v_, now)
        lib.orc_ip_colocation(v_)
        lib.orc_compute_scores(v_)
        gpu = ob.NetState(net, params, thresholds=beacon_thresholds(), p5=p5, ip_white=white)
        gpu.pull_from_engine(eng)
        assert_state_equal(st, gpu, ["estate", "p6", "score"])
        assert np.array_equal(bits(eng.scores()), bits(st.score))
    hub = st.p6[row_ptr[0]:row_ptr[1]]          # (NetState fields are in edge order)
    assert (hub > 0).sum() > 100, "the hub's shared IPs are counted"
    eng.close()