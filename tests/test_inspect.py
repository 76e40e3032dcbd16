"""Score inspection and IP refresh through the C ABI, against the oracle:
gsim_read_snapshot is WithPeerScoreInspect's ExtendedPeerScoreInspectFn view
(score.go:127-180, inspectScoresExtended 472-500) and gsim_set_ips is
refreshIPs (score.go:568-585)."""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second

from test_heartbeat import SEED, assert_same, tick_time
from test_delivery import R, T0


def test_snapshot_layout_matches_header():
    # gsim.h: 4 doubles + 2 u32 + 2 i32 = 48 bytes; i64 + 3 doubles = 32 bytes
    assert np.dtype(_abi.PEER_SNAPSHOT_DTYPE).itemsize == 48
    assert np.dtype(_abi.TOPIC_SNAPSHOT_DTYPE).itemsize == 32


def _setup(n=1500, k=16, T=3, seed=12, shards=0):
    from fixtures import beacon_params, sybil_ips, synthetic_state
    from gsim.engine import Engine, random_regular
    from gsim.shard import ShardedEngine
    rng = np.random.default_rng(seed)
    net = random_regular(n, k, seed=seed, n_topics=T)
    net.ip_ptr, net.ip_ids, net.n_ips = sybil_ips(n, 0.2, 4, rng)
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    p5 = rng.normal(0, 3, n)
    st = ob.NetState(net, params, thresholds=th, gossip=gp, p5=p5)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    st.estate[rng.random(net.e) < 0.03] = 0                   # some untracked edges
    eng = ShardedEngine(params, th, gossip=gp, shards=shards) if shards else Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_app_score(p5)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    return rng, net, params, th, gp, p5, st, eng


def _check_snapshot(eng, st, net, p5, lo, hi):
    peers, topics = eng.snapshot(lo, hi)
    e0, e1 = int(net.row_ptr[lo]), int(net.row_ptr[hi])
    sl = slice(e0, e1)
    owner = net.owner()
    tracked = (st.estate[sl] & _abi.ES_TRACKED) != 0
    assert (peers["tracked"] == tracked).all()
    assert (peers["observer"] == owner[sl]).all() and (peers["peer"] == net.col[sl]).all()
    exp_score = np.where(tracked, st.score[sl], 0.0)
    assert np.array_equal(peers["score"].view(np.uint64), exp_score.view(np.uint64))
    assert np.array_equal(peers["app_specific_score"], np.where(tracked, p5[net.col[sl]], 0.0))
    assert np.array_equal(peers["ip_colocation_factor"], np.where(tracked, st.p6[sl], 0.0))
    assert np.array_equal(peers["behaviour_penalty"], np.where(tracked, st.bp[sl], 0.0))
    in_mesh = (st.tflags[:, sl] & _abi.TF_IN_MESH) != 0
    tm = np.where(in_mesh & tracked[None, :], st.mesh_time[:, sl], 0).T
    assert np.array_equal(topics["time_in_mesh_ns"], tm)
    for f, name in (("first", "first_message_deliveries"), ("meshd", "mesh_message_deliveries"),
                    ("invalid", "invalid_message_deliveries")):
        exp = np.where(tracked[None, :], getattr(st, f)[:, sl], 0.0).T
        assert np.array_equal(topics[name], exp), name


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [0, 3])
def test_snapshot_after_refresh_and_live_after_deliveries(require_gpu, shards):
    """Right after a refresh the snapshot's scores are the score snapshot;
    after a tick of deliveries they are the live score (the oracle's counters
    already hold every delivery), meshMessageDeliveries pending increments
    included.  On 3 shards through the group readback (gsim_group_read_snapshot,
    gsim_group_read_scores): observer ranges that cross shard bounds."""
    rng, net, params, th, gp, p5, st, eng = _setup(shards=shards)
    lib = ob.load()
    now = tick_time(1)
    eng.refresh_scores(now)
    v = st.view()
    lib.orc_refresh_scores(v, now)
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    _check_snapshot(eng, st, net, p5, 0, net.n)
    _check_snapshot(eng, st, net, p5, 100, 117)
    if shards:
        b = eng.bounds
        _check_snapshot(eng, st, net, p5, int(b[1]) - 7, int(b[2]) + 5)   # across two bounds
        assert np.array_equal(eng.scores().view(np.uint64), st.score.view(np.uint64))
    # a tick of propagation: deliveries change counters after the snapshot
    from test_delivery import _schedule
    msgs = ob.Msgs(net.n, st.T, 256, R, T0, Second)
    eng.msgs_init(256, R, T0, Second)
    eng.heartbeat(1, now)
    msgs.heartbeat(st, 1, now, SEED)
    sched = _schedule(rng, [1], st.T, R, 12, 0.1, net.n)
    for g in range(R, 2 * R):
        for (mid, t, o, inv) in sched.get(g, []):
            msgs.publish(st, mid, t, o, inv, g)
        if g in sched:
            eng.publish(sched[g], g)
        msgs.round(st, g)
        eng.round(g)
    assert msgs.stats[0] > 0
    snap_before = st.score.copy()
    lib.orc_compute_scores(st.view())             # live scores of the oracle state
    assert not np.array_equal(snap_before, st.score), "deliveries moved some scores"
    _check_snapshot(eng, st, net, p5, 0, net.n)
    eng.close()


@pytest.mark.gpu
def test_set_ips_rederives_colocation(require_gpu):
    """refreshIPs: a fifth of the peers move to other (partly shared)
    addresses; P6 and the scores after the next refresh match the oracle's."""
    rng, net, params, th, gp, p5, st, eng = _setup(seed=19)
    lib = ob.load()
    now = tick_time(1)
    eng.refresh_scores(now)
    v = st.view()
    lib.orc_refresh_scores(v, now)
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    # new addresses: 20 % of the peers onto a pool of 30 ids, some with two
    n = net.n
    lists = [list(net.ip_ids[net.ip_ptr[i]:net.ip_ptr[i + 1]]) for i in range(n)]
    n_ips = net.n_ips + 30
    for i in rng.choice(n, n // 5, replace=False):
        lists[i] = [net.n_ips + int(rng.integers(0, 30))]
        if rng.random() < 0.3:
            lists[i].append(net.n_ips + int(rng.integers(0, 30)))
            lists[i] = sorted(set(lists[i]))
    ip_ptr = np.concatenate([[0], np.cumsum([len(x) for x in lists])]).astype(np.uint32)
    ip_ids = np.array([x for l in lists for x in l], dtype=np.uint32)
    eng.set_ips(ip_ptr, ip_ids, n_ips)
    net.ip_ptr, net.ip_ids, net.n_ips = ip_ptr, ip_ids, n_ips
    now = tick_time(2)
    eng.refresh_scores(now)
    v = st.view()
    lib.orc_refresh_scores(v, now)
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    gpu = ob.NetState(net, params, thresholds=th, gossip=gp, p5=p5)
    gpu.pull_from_engine(eng)
    assert_same(st, gpu)
    assert (st.p6 > 0).sum() > 0
    eng.close()
