"""Heartbeat mesh maintenance + GRAFT/PRUNE handling.

CPU part: behavioural invariants of the oracle restatement, mirroring what the
reference's integration tests assert (gossipsub_test.go: mesh sizes, the
negative-score sinkhole 1526-1608, backoff 585-681, opportunistic grafting
1804-1916).  GPU part: the engine's heartbeat/control kernels against the
oracle, bit-exact on every state array, over many ticks.
"""
import numpy as np
import pytest

import oracle_binding as ob
from fixtures import beacon_params, beacon_thresholds, randomize_state
from gsim import _abi
from gsim.engine import Engine, random_regular
from gsim.params import GossipSubParams, PeerScoreParams, PeerScoreThresholds, Second, TopicScoreParams

SEED = 0x1234_5678_9ABC_DEF0
HB = Second


def tick_time(k):
    return 1000 * Second + k * HB


def mesh(st):
    return (st.tflags & _abi.TF_MESH) != 0


def run_tick_oracle(st, k, refresh=True):
    lib = ob.load()
    v = st.view()
    now = tick_time(k)
    if refresh:
        lib.orc_refresh_scores(v, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
    lib.orc_heartbeat(v, k, now, SEED)
    lib.orc_handle_control(v, 0, now + HB // 11)
    lib.orc_handle_control(v, 1, now + 2 * HB // 11)


def simple_params(T=1, p5=None):
    tp = TopicScoreParams(TopicWeight=1, TimeInMeshWeight=0.01, TimeInMeshQuantum=Second, TimeInMeshCap=10,
                          FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=0.5,
                          FirstMessageDeliveriesCap=10, InvalidMessageDeliveriesWeight=-1,
                          InvalidMessageDeliveriesDecay=0.5)
    p = PeerScoreParams(AppSpecificScore=(lambda q: p5[q]) if p5 is not None else (lambda q: 0.0),
                        AppSpecificWeight=1, DecayInterval=Second, DecayToZero=0.01)
    for t in range(T):
        p.Topics[f"t{t}"] = tp
    return p


def new_state(n, k, T, params, gp=None, th=None, seed=1, p5=None):
    net = random_regular(n, k, seed=seed, n_topics=T)
    st = ob.NetState(net, params, thresholds=th or PeerScoreThresholds(), gossip=gp or GossipSubParams(),
                     p5=p5)
    return net, st


# ---- oracle behaviour -----------------------------------------------------------

def test_first_heartbeat_fills_meshes_to_D():
    """From empty meshes every peer grafts D peers (gossipsub.go:1413-1427)."""
    net, st = new_state(400, 20, 1, simple_params(), gp=GossipSubParams(D=6, Dlo=5, Dhi=12))
    lib = ob.load()
    v = st.view()
    lib.orc_compute_scores(v)
    lib.orc_heartbeat(v, 1, tick_time(1), SEED)
    m = mesh(st)[0]
    starts = net.row_ptr[:-1].astype(np.int64)
    deg = np.add.reduceat(m.astype(np.int64), starts)
    outb = np.add.reduceat((m & (net.outbound != 0)).astype(np.int64), starts)
    # D from the Dlo graft, then the Dout top-up adds outbound peers (1492-1518)
    assert (deg >= 6).all() and (deg <= 6 + 2).all()
    assert ((deg == 6) | (outb == 2)).all()
    assert (outb >= 2).all()
    grafts = (st.ctl[0, 0] & _abi.CTL_GRAFT) != 0
    assert grafts.sum() == deg.sum()                    # one GRAFT per new mesh link
    assert ((st.tflags[0] & _abi.TF_IN_MESH) != 0).sum() == deg.sum()   # tracer.Graft


def test_mesh_symmetric_and_bounded_after_control_rounds():
    gp = GossipSubParams(D=6, Dlo=5, Dhi=12)
    net, st = new_state(500, 20, 2, simple_params(2), gp=gp)
    for k in range(1, 6):
        run_tick_oracle(st, k)
        m = mesh(st)
        rev = st.rev
        for t in range(2):
            assert np.array_equal(m[t], m[t][rev]), "mesh must be symmetric after GRAFT/PRUNE exchange"
        assert not st.ctl.any(), "all control records consumed"
        deg = np.add.reduceat(m[0].astype(np.int64), net.row_ptr[:-1].astype(np.int64))
        assert deg.min() >= 1 and deg.max() <= 20


def test_negative_score_sinkhole_never_in_mesh():
    """gossipsub_test.go:1526-1608: a peer with AppSpecificScore -1000 is pruned
    and never (re)grafted, by heartbeat or by handleGraft."""
    n = 300
    p5 = np.zeros(n)
    p5[0] = -1000.0
    params = simple_params(1, p5=p5)
    net, st = new_state(n, 16, 1, params, gp=GossipSubParams(D=6, Dlo=5, Dhi=12), p5=p5)
    # peer 0 starts inside everybody's mesh
    st.tflags[0, :] |= (st.net.col == 0).astype(np.uint8) * _abi.TF_MESH
    for k in range(1, 8):
        run_tick_oracle(st, k)
        m = mesh(st)[0]
        assert not m[st.net.col == 0].any(), f"tick {k}: sinkholed peer in a mesh"


def test_backoff_blocks_regraft_and_is_cleared_on_tick15():
    """gossipsub.go:1412-1421 skips backed-off peers; clearBackoff (1627-1646)
    drops entries 2s past expiry on 15-tick boundaries only."""
    gp = GossipSubParams(D=6, Dlo=5, Dhi=12, PruneBackoff=5 * Second)
    net, st = new_state(200, 12, 1, simple_params(), gp=gp)
    st.backoff[0, :] = tick_time(0) + 3 * Second       # every link backed off until tick 3
    lib = ob.load()
    v = st.view()
    lib.orc_compute_scores(v)
    lib.orc_heartbeat(v, 1, tick_time(1), SEED)
    assert not mesh(st).any(), "backoff existence blocks grafting"
    lib.orc_heartbeat(v, 14, tick_time(14), SEED)
    assert not mesh(st).any()
    lib.orc_heartbeat(v, 15, tick_time(15), SEED)       # cleared (expired + 2s < now), then grafted
    assert mesh(st).any()


def test_opportunistic_graft_only_on_tick_multiple():
    """gossipsub.go:1520-1552 every OpportunisticGraftTicks when median < threshold."""
    gp = GossipSubParams(D=4, Dlo=3, Dhi=8, OpportunisticGraftTicks=60, OpportunisticGraftPeers=2)
    th = PeerScoreThresholds(OpportunisticGraftThreshold=1.0)
    net, st = new_state(200, 16, 1, simple_params(), gp=gp, th=th)
    lib = ob.load()
    v = st.view()
    lib.orc_compute_scores(v)
    lib.orc_heartbeat(v, 1, tick_time(1), SEED)          # fill to D=4 with score-0 peers
    st.ctl[...] = 0
    # give every non-mesh peer a better score than the (all-zero) mesh median
    st.score[~mesh(st)[0]] = 5.0
    before = mesh(st)[0].copy()
    starts = net.row_ptr[:-1].astype(np.int64)
    lib.orc_heartbeat(v, 59, tick_time(59), SEED)
    assert np.array_equal(before, mesh(st)[0])
    lib.orc_heartbeat(v, 60, tick_time(60), SEED)
    grew = np.add.reduceat(mesh(st)[0].astype(np.int64), starts) - np.add.reduceat(before.astype(np.int64), starts)
    assert (grew == 2).all()                          # OpportunisticGraftPeers better-than-median peers
    assert (st.score[mesh(st)[0] & ~before] == 5.0).all()


def test_dhi_prune_keeps_dscore_best_and_dout_outbound():
    """gossipsub.go:1429-1490: an oversubscribed mesh is cut to D, keeping the
    Dscore best-scoring peers and at least Dout outbound peers."""
    gp = GossipSubParams(D=6, Dlo=5, Dhi=8, Dscore=3, Dout=2)
    net, st = new_state(100, 20, 1, simple_params(), gp=gp)
    rng = np.random.default_rng(4)
    st.tflags[0, :] = _abi.TF_MESH                      # everyone in every mesh (20 > Dhi)
    st.score[:] = rng.integers(0, 5, size=net.e).astype(np.float64)
    lib = ob.load()
    v = st.view()
    lib.orc_heartbeat(v, 1, tick_time(1), SEED)
    for i in range(net.n):
        b, e = int(net.row_ptr[i]), int(net.row_ptr[i + 1])
        m = mesh(st)[0][b:e]
        assert m.sum() == gp.D
        s = st.score[b:e]
        kept = np.sort(s[m])[::-1]
        assert (kept[:gp.Dscore] == np.sort(s)[::-1][:gp.Dscore]).all()
        if net.outbound[b:e].sum() >= gp.Dout:
            assert net.outbound[b:e][m].sum() >= gp.Dout


def test_graft_into_backoff_gets_penalty_and_prune():
    """gossipsub.go:780-798 (and gossipsub_spam_test.go:365-600): a GRAFT while
    backing off costs P7 1 (2 under the flood cutoff), refreshes backoff, PRUNE back."""
    gp = GossipSubParams(D=6, Dlo=5, Dhi=12, PruneBackoff=60 * Second, GraftFloodThreshold=10 * Second)
    net, st = new_state(50, 10, 1, simple_params(), gp=gp)
    lib = ob.load()
    v = st.view()
    now = tick_time(5)
    e = int(net.row_ptr[3])                 # receiver 3's first connection
    st.backoff[0, e] = now + 55 * Second    # pruned 5s ago: inside the flood cutoff
    st.ctl[0, 0, e] = _abi.CTL_GRAFT
    lib.orc_handle_control(v, 0, now)
    assert st.bp[e] == 2.0
    assert st.backoff[0, e] == now + 60 * Second
    assert st.ctl[1, 0, st.rev[e]] & _abi.CTL_PRUNE
    assert not mesh(st)[0, e]
    st.ctl[...] = 0
    st.backoff[0, e] = now + 45 * Second    # pruned 15s ago: past the flood cutoff
    st.ctl[0, 0, e] = _abi.CTL_GRAFT
    lib.orc_handle_control(v, 0, now)
    assert st.bp[e] == 3.0


# ---- GPU parity -------------------------------------------------------------------

def _random_mesh_state(st, rng, p_mesh):
    st.tflags[...] |= (rng.random(st.tflags.shape) < p_mesh).astype(np.uint8) * _abi.TF_MESH
    bo = rng.random(st.backoff.shape)
    st.backoff[...] = np.where(bo < 0.05, tick_time(0) + rng.integers(-10, 120, st.backoff.shape) * Second, 0)


def assert_same(cpu, gpu):
    for f in cpu.TOPIC_FIELDS + cpu.EDGE_FIELDS + ("ctl", "lastpub", "fan_topics"):
        a, b = getattr(cpu, f), getattr(gpu, f)
        av = a.view(np.uint64) if a.dtype.itemsize == 8 else a
        bv = b.view(np.uint64) if b.dtype.itemsize == 8 else b
        if not np.array_equal(av, bv):
            bad = np.argwhere(av != bv)
            idx = tuple(bad[0])
            raise AssertionError(f"{f}: {len(bad)} mismatches, first {idx}: cpu={a[idx]!r} gpu={b[idx]!r}")


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,T,p_mesh,ticks", [
    (500, 16, 1, 0.0, [1, 2, 3]),            # empty start: Dlo grafting, GRAFT acceptance
    (1200, 32, 3, 0.55, [14, 15, 16]),       # oversubscribed: Dhi prune + Dout rotation, clearBackoff
    (800, 24, 2, 0.3, [59, 60, 61]),         # opportunistic grafting tick
    (600, 16, 2, 0.85, [1, 2, 3]),           # Dhi prune on short rows (16 connections)
    (300, 64, 1, 0.3, [4, 5]),               # full-wave rows (64 connections)
    (700, 16, 3, 0.45, [59, 60]),            # four observers per wavefront: opportunistic tick, Dhi prune
    (900, 12, 20, 0.6, [14, 15]),            # 16-lane groups, 20 topics (lastput words of topics gl, gl+16)
])
def test_heartbeat_and_control_bit_exact(require_gpu, n, k, T, p_mesh, ticks):
    rng = np.random.default_rng(n + T)
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, OpportunisticGraftTicks=60)
    th = PeerScoreThresholds(GossipThreshold=-100, PublishThreshold=-200, GraylistThreshold=-300,
                             OpportunisticGraftThreshold=3.0)
    net = random_regular(n, k, seed=n, n_topics=T)
    p5 = np.where(rng.random(n) < 0.08, -50.0, np.round(rng.normal(0, 3, n)))   # ties + negatives
    st = ob.NetState(net, params, thresholds=th, gossip=gp, p5=p5)
    randomize_state(st, rng, tick_time(0), retained_frac=0.0)
    _random_mesh_state(st, rng, p_mesh)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_app_score(p5)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    for kk in ticks:
        now = tick_time(kk)
        eng.refresh_scores(now)
        eng.heartbeat(kk, now)
        eng.handle_control(0, now + HB // 11)
        eng.handle_control(1, now + 2 * HB // 11)
        run_tick_oracle(st, kk)
        gpu = ob.NetState(net, params, thresholds=th, gossip=gp, p5=p5)
        gpu.pull_from_engine(eng)
        assert_same(st, gpu)
    eng.close()


@pytest.mark.gpu
def test_lazy_mesh_time_unread_ticks(require_gpu):
    """Lazy meshTime: the refresh no longer stores meshTime;
    scores, PRUNE freezes, churn and the read-out derive it from graftTime and
    the last refresh's clock.  Several ticks with churn and no read in between,
    then a heartbeat whose clock runs backwards, must leave every array (the
    scores included) bit-exact against the oracle, which stores it."""
    n, k, T = 1000, 24, 2
    rng = np.random.default_rng(77)
    params = beacon_params(T)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, OpportunisticGraftTicks=60)
    th = PeerScoreThresholds(GossipThreshold=-100, PublishThreshold=-200, GraylistThreshold=-300,
                             OpportunisticGraftThreshold=3.0)
    net = random_regular(n, k, seed=n, n_topics=T)
    p5 = np.where(rng.random(n) < 0.08, -50.0, np.round(rng.normal(0, 3, n)))
    st = ob.NetState(net, params, thresholds=th, gossip=gp, p5=p5)
    randomize_state(st, rng, tick_time(0), retained_frac=0.0)
    _random_mesh_state(st, rng, 0.55)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_app_score(p5)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    src = net.owner()
    und = np.nonzero(src < net.col)[0]
    down = np.stack([src[und], net.col[und]], 1)[rng.random(len(und)) < 0.03].astype(np.uint32)
    lib = ob.load()
    try:
        for kk in range(58, 64):
            now = tick_time(kk)
            if kk == 60:
                eng.set_connections(down, up=False, now=now - HB // 2)
                st.churn(down, up=False, now=now - HB // 2)
            if kk == 62:
                eng.set_connections(down, up=True, now=now - HB // 2)
                st.churn(down, up=True, now=now - HB // 2)
            eng.refresh_scores(now)
            eng.heartbeat(kk, now)
            eng.handle_control(0, now + HB // 11)
            eng.handle_control(1, now + 2 * HB // 11)
            run_tick_oracle(st, kk)
        # the clock runs backwards: a heartbeat before the last refresh's time
        back = tick_time(63) - 3 * HB
        eng.heartbeat(64, back)
        eng.handle_control(0, back + HB // 11)
        lib.orc_heartbeat(st.view(), 64, back, SEED)
        lib.orc_handle_control(st.view(), 0, back + HB // 11)
        eng.compute_scores()
        lib.orc_compute_scores(st.view())
        gpu = ob.NetState(net, params, thresholds=th, gossip=gp, p5=p5)
        gpu.pull_from_engine(eng)
        assert_same(st, gpu)
        assert ((st.tflags & _abi.TF_IN_MESH) != 0).any() and (st.mesh_time > 0).any()
    finally:
        eng.close()


def _go_dout_keep(plst, outbound, D, Dout):
    """gossipsub.go:1457-1488 verbatim: returns plst[:D] after the rotation."""
    plst = list(plst)
    ob = sum(1 for p in plst[:D] if outbound[p])
    if ob < Dout:
        def rotate(i):
            p = plst[i]
            for j in range(i, 0, -1):
                plst[j] = plst[j - 1]
            plst[0] = p
        if ob > 0:
            ihave = ob
            i = 1
            while i < D and ihave > 0:
                if outbound[plst[i]]:
                    rotate(i)
                    ihave -= 1
                i += 1
        ineed = Dout - ob
        i = D
        while i < len(plst) and ineed > 0:
            if outbound[plst[i]]:
                rotate(i)
                ineed -= 1
            i += 1
    return set(plst[:D])


def _closed_form_keep(plst, outbound, D, Dout):
    """The data-parallel form k_heartbeat evaluates per lane (heartbeat.hip)."""
    pos = {p: i for i, p in enumerate(plst)}
    inD = {p for p in plst if pos[p] < D}
    obD = sum(1 for p in inD if outbound[p])
    if obD >= Dout:
        return inD
    rest = {p for p in inD if not (outbound[p] and pos[p] >= 1)}
    cb = sorted((p for p in plst if pos[p] >= D and outbound[p]), key=lambda p: pos[p])
    j = min(Dout - obD, len(cb))
    rest_sorted = sorted(rest, key=lambda p: pos[p])
    pushed = set(rest_sorted[len(rest_sorted) - j:]) if j else set()
    return (inD - pushed) | set(cb[:j])


def test_dout_rotation_closed_form_matches_go():
    rng = np.random.default_rng(7)
    for _ in range(20000):
        D = int(rng.integers(2, 12))
        Dout = int(rng.integers(0, D // 2 + 1))
        l = int(rng.integers(D + 1, 40))
        plst = list(rng.permutation(64)[:l])
        outbound = {p: bool(rng.random() < rng.random()) for p in plst}
        assert _go_dout_keep(plst, outbound, D, Dout) == _closed_form_keep(plst, outbound, D, Dout)
