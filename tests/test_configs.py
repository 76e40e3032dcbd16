"""Parity at the shapes of BASELINE.json's configurations (SURVEY.md §8 table
C1-C5), scaled to sizes the oracle finishes in seconds.  C3 itself is the
bench workload (bench.py); its structure (random-regular k=32, 16 topics,
beacon params) is covered by test_delivery/test_gossip.

  C1  Go mocknet-like: 100 hosts, dense (k=20), 1 topic, D=6 defaults,
      1000 messages
  C2  10k peers, single topic, D=8, full P1-P7 + gossip (full size)
  C4  Sybil/eclipse: 20 % sybils behind shared IPs, sybils ignore IWANT
      (broken promises -> P7), P6 colocation, opportunistic grafting tick
  C5  power-law graph (Chung-Lu, exponent 2.5, mean 16, rows <= 64), 64
      topics with Zipf subscriptions (~8 per peer), churn between ticks
"""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second

from test_heartbeat import tick_time


def test_power_law_graph_shape():
    from gsim import graphs
    net = graphs.power_law(20000, 16, 2.5, 64, seed=4)
    d = np.diff(net.row_ptr.astype(np.int64))
    assert d.max() <= 64 and 12 < d.mean() < 17
    assert d.max() >= 48, "heavy tail up to the row cap"
    assert (net.col[net.rev()] == net.owner()).all(), "symmetric"
    rows_sorted = all((np.diff(net.col[a:b].astype(np.int64)) > 0).all()
                      for a, b in zip(net.row_ptr[:-1:97], net.row_ptr[1::97]))
    assert rows_sorted
    ob_ = net.outbound.astype(np.int64) + net.outbound[net.rev()].astype(np.int64)
    assert (ob_ == 1).all(), "exactly one side dialed"


def test_zipf_subscriptions():
    from gsim import graphs
    sub = graphs.zipf_subscriptions(50000, 64, 8, seed=1)
    per_peer = np.array([bin(int(x)).count("1") for x in sub[:1000]])
    assert (per_peer == 8).all()
    cnt = [int(((sub >> np.uint64(t)) & np.uint64(1)).sum()) for t in range(64)]
    assert cnt[0] > cnt[10] > cnt[63] > 0, "popularity falls with rank"


def test_sybil_ips():
    from gsim import graphs
    ip_ptr, ip_ids, n_ips, syb = graphs.sybil_ips(12500, 0.2, 50, seed=1)
    assert syb.sum() == 2500 and n_ips == 10000 + 50
    _, counts = np.unique(ip_ids[syb], return_counts=True)
    assert (counts == 50).all()


# ---- GPU parity -------------------------------------------------------------------

@pytest.mark.gpu
def test_c1_mocknet_dense_default_params(require_gpu):
    """C1: 100 hosts, k=20, 1 topic, D=6 and the library's default
    GossipSubParams, 1000 messages over 20 heartbeats."""
    from gsim.engine import random_regular
    from tickrun import run_parity, subscribed_schedule
    from test_delivery import delivery_params
    rng = np.random.default_rng(101)
    net = random_regular(100, 20, seed=5, n_topics=1)
    params = delivery_params(1)
    th = PeerScoreThresholds(GossipThreshold=-10, PublishThreshold=-50, GraylistThreshold=-80)
    gp = GossipSubParams()                                    # D=6, Dlo=5, Dhi=12, Dlazy=6, ...
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    ticks = list(range(1, 21))
    sched = subscribed_schedule(rng, ticks, net, 1, 50, 0.02)
    n_msgs = sum(len(v) for v in sched.values())
    assert 850 <= n_msgs <= 1150
    msgs, _ = run_parity(net, params, th, gp, st, ticks, sched, ring=1024)
    assert msgs.stats[1] > 0.95 * n_msgs * 99, "messages reach (nearly) every host"


@pytest.mark.gpu
def test_c2_10k_single_topic_full_scoring(require_gpu):
    """C2 at full size: 10k peers, k=32, one topic, D=8, P1-P7 + gossip."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from tickrun import run_parity, subscribed_schedule
    rng = np.random.default_rng(202)
    net = random_regular(10_000, 32, seed=7, n_topics=1)
    params = beacon_params(1)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / 32)
    st.bp[rng.random(net.e) < 0.03] = 12.0
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, 1, 8, 0.05)
    _, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=256)
    assert gs["iwant_ids"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_c3_shape_from_device_fill(require_gpu):
    """C3's shape at 20k peers: random-regular k=32, 16 topics, the bench's
    beacon-style params and thresholds, starting from gsim_fill_synthetic
    (the state bench.py runs from), 5 ticks at 4 msg/s/topic with 2 % invalid
    messages: mesh maintenance, control, gossip and promises, every array
    bit-exact against the oracle after each tick."""
    from fixtures import beacon_params, beacon_thresholds
    from gsim.engine import Engine, random_regular
    from tickrun import SEED, run_parity, subscribed_schedule
    rng = np.random.default_rng(303)
    n, T = 20_000, 16
    net = random_regular(n, 32, seed=17, n_topics=T)
    params = beacon_params(T)
    th = beacon_thresholds()
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_seed(SEED)
    eng.fill_synthetic(seed=31, now=tick_time(0), p_mesh=8 / 32)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    st.pull_from_engine(eng)
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.02)
    msgs, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=1024, eng=eng)
    assert gs["iwant_ids"] > 0 and msgs.stats[3] >= 0
    assert msgs.stats[0] == msgs.stats[1] + msgs.stats[2]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_c3_full_size_invariants(require_gpu):
    """The bench workload itself (1M peers, k=32, 16 topics, beacon params,
    4 msg/s/topic) for 3 ticks, checked through size-independent properties:
      * right after the heartbeat every (peer, topic) mesh has <= Dhi + Dout
        members (a mesh at Dhi is not pruned, and the Dout top-up,
        gossipsub.go:1492-1518, may then add Dout outbound peers); in the
        first tick some mesh goes above Dhi that way;
      * every mesh link that changed between the start of a tick and the end
        of its control rounds (GRAFT/PRUNE and their replies) ends symmetric;
      * accepted deliveries = first + duplicate, and no error (queue overflow,
        early slot reuse) is reported."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    cfg = bench.CONFIGS["c3"]
    eng, net = bench.build_engine(cfg, seed=1, device=0)
    n, T, Dhi = cfg[0], cfg[2], cfg[5]
    Dout = 2                                   # GossipSubParams default, bench.build_engine
    rev = net.rev()
    rp = net.row_ptr.astype(np.int64)
    sched = bench.message_schedule(n, T, range(1, 4), seed=2)
    try:
        def mesh():
            return (eng.read(_abi.F_TFLAGS) & _abi.TF_MESH) != 0
        before = mesh()
        for k in range(1, 4):
            now = bench.tick_time(k)
            eng.refresh_scores(now)
            eng.heartbeat(k, now)
            after_hb = mesh()
            top = 0
            for t in range(T):
                sizes = np.add.reduceat(after_hb[t].astype(np.int32), rp[:-1])
                assert sizes.max() <= Dhi + Dout, f"tick {k} topic {t}: mesh above Dhi + Dout after the heartbeat"
                top = max(top, int(sizes.max()))
            assert top > Dhi or k > 1, "a mesh at Dhi short of outbound peers is topped up"
            del after_hb
            for g in range(k * bench.ROUNDS, (k + 1) * bench.ROUNDS):
                if g in sched:
                    eng.publish_array(sched[g], g)
                eng.round(g)
                if g == k * bench.ROUNDS + 1:
                    final = mesh()
                    changed = before != final
                    assert changed.any(), "the heartbeat changed some links"
                    for t in range(T):
                        c = np.nonzero(changed[t])[0]
                        assert np.array_equal(final[t][c], final[t][rev[c]]), f"tick {k} topic {t}: asymmetric"
                    del changed
            before = mesh()
            st = eng.msg_stats()
            assert st[0] == st[1] + st[2] and st[1] > 0
    finally:
        eng.close()


@pytest.mark.gpu
def test_c4_sybil_colocation_broken_promises(require_gpu):
    """C4 scaled 1/10: 10k honest + 2.5k sybils that never answer IWANT.  The
    sybils sit behind few addresses (500 per IP), so an honest peer sees several
    of its neighbours on one IP: P6 colocation pushes them below the publish and
    graylist thresholds, broken promises add P7; ticks 58-61 include the
    opportunistic-grafting heartbeat."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from gsim.engine import random_regular
    from tickrun import run_parity, subscribed_schedule
    rng = np.random.default_rng(404)
    n = 12_500
    net = random_regular(n, 32, seed=9, n_topics=1)
    ip_ptr, ip_ids, n_ips, syb = graphs.sybil_ips(n, 0.2, 500, seed=3)
    net = graphs.with_ips(net, ip_ptr, ip_ids, n_ips)
    params = beacon_params(1)
    th = PeerScoreThresholds(GossipThreshold=-100, PublishThreshold=-500, GraylistThreshold=-1000,
                             AcceptPXThreshold=100, OpportunisticGraftThreshold=5)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, OpportunisticGraftTicks=60)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(57), 8 / 32)
    beh = syb.astype(np.uint8) * ob.ORC_BEHAVE_IGNORE_IWANT
    ticks = [58, 59, 60, 61]
    sched = subscribed_schedule(rng, ticks, net, 1, 10, 0.0)
    seen_p6 = {}

    def check(kk, st_, msgs):
        if kk == 58:
            seen_p6["sybil"] = st_.p6[syb[net.col]]
            seen_p6["graylisted"] = int((st_.score[syb[net.col]] < th.GraylistThreshold).sum())

    run_parity(net, params, th, gp, st, ticks, sched, ring=256, behaviour=beh, after_tick=check)
    assert (seen_p6["sybil"] > 0).mean() > 0.2, "many views of a sybil carry P6"
    assert seen_p6["graylisted"] > 0, "some sybils are graylisted"


@pytest.mark.gpu
@pytest.mark.parametrize("topic_slots", [0, 16])
def test_c5_power_law_zipf_topics_churn(require_gpu, topic_slots):
    """C5 scaled: power-law graph (rows up to 64), 64 topics with Zipf
    subscriptions (~8 per peer), connections churning between ticks,
    publishers outside a topic using fanout (their topic slots and, with
    per-topic sub-rings, the topics' member-compacted seen-set cells grow at
    publication).  topic_slots: 0 = one shared ring, 16 = sub-rings."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from tickrun import restrict_to_subscriptions, run_parity, subscribed_schedule
    rng = np.random.default_rng(505)
    n, T = 3000, 64
    net = graphs.power_law(n, 16, 2.5, 64, seed=11, n_topics=T)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 8, seed=12))
    params = beacon_params(T, RetainScore=3 * Second)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.3)
    restrict_to_subscriptions(st, net)
    ticks = list(range(1, 7))
    sched = subscribed_schedule(rng, ticks, net, T, 1.0, 0.02, member_only=False)
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    pick = lambda k: und[rng.choice(len(und), size=len(und) // 50, replace=False)]  # noqa: E731
    downs = {k: pick(k) for k in (2, 4)}
    churn = {2: [(downs[2], False)], 4: [(downs[2], True), (downs[4], False)], 6: [(downs[4], True)]}
    run_parity(net, params, th, gp, st, ticks, sched, ring=1024, churn=churn, topic_slots=topic_slots)
    assert (np.diff(net.row_ptr.astype(np.int64)) > 32).any(), "rows longer than half a wave"


@pytest.mark.gpu
@pytest.mark.parametrize("topic_slots", [0, 64])
@pytest.mark.parametrize("width", [8, 16, 32, 64])
def test_ihave_lane_widths_bit_exact(require_gpu, width, topic_slots):
    """The IHAVE/IWANT walk (k_ihave) with 8-, 16-, 32- and 64-lane row groups on
    one power-law graph (rows of 1-64 connections: a narrow group walks the
    long rows in chunks): every width is bit-exact against the oracle, so
    all give the same promises, IWANT ids and responses.  topic_slots 64:
    sub-rings, the member-major walk with the window masks."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from gsim.engine import Engine
    from tickrun import SEED, restrict_to_subscriptions, run_parity, subscribed_schedule
    rng = np.random.default_rng(707)
    n, T = 2500, 8
    net = graphs.power_law(n, 16, 2.5, 64, seed=21, n_topics=T)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 3, seed=22))
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
    gp = GossipSubParams(D=6, Dlo=4, Dhi=10, Dscore=3, Dout=2)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.25)
    restrict_to_subscriptions(st, net)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    eng.set_kernel_variant(3, width)
    ticks = list(range(1, 5))
    sched = subscribed_schedule(rng, ticks, net, T, 3.0, 0.02)
    _, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=512, eng=eng, topic_slots=topic_slots)
    assert gs["iwant_ids"] > 0 and (np.diff(net.row_ptr.astype(np.int64)) > 32).any()


@pytest.mark.gpu
def test_c5_from_device_fill_skips_unjoined_records(require_gpu):
    """Start from gsim_fill_synthetic (records only where both endpoints
    joined the topic), the state bench.py's c5 runs from: the score pass then
    skips every record of a topic its observer did not join.  Ticks with
    churn, fanout publishers and gossip stay bit-exact against the oracle,
    which reads every record."""
    from gsim import graphs
    from gsim.engine import Engine
    from fixtures import beacon_params
    from tickrun import SEED, run_parity, subscribed_schedule
    rng = np.random.default_rng(606)
    n, T = 3000, 64
    net = graphs.power_law(n, 16, 2.5, 64, seed=13, n_topics=T)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 8, seed=14))
    params = beacon_params(T, RetainScore=3 * Second)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second)
    eng = Engine(params, th, gossip=gp)
    eng.load_graph(net)
    eng.set_seed(SEED)
    eng.fill_synthetic(seed=77, now=tick_time(0), p_mesh=0.5)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    st.pull_from_engine(eng)
    joined = ((net.sub[net.owner()][None, :] >> np.arange(T, dtype=np.uint64)[:, None]) & np.uint64(1)) != 0
    assert (st.first[~joined] == 0).all() and (st.first[joined] != 0).any()
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 1.0, 0.02, member_only=False)
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 50, replace=False)]
    churn = {2: [(down, False)], 4: [(down, True)]}
    run_parity(net, params, th, gp, st, ticks, sched, ring=1024, churn=churn, eng=eng)


@pytest.mark.gpu
@pytest.mark.parametrize("topic_slots", [0, 32])
def test_hub_rows_bit_exact(require_gpu, topic_slots):
    """Hub observers (rows of 65-1024 connections, SURVEY §8 C5's power law
    with its cap raised): the heartbeat, fanout maintenance and fanout
    publication of hubs run one block per observer (BlockGroup), control
    handling walks long rows in 64-edge chunks, delivery uses the flattened
    topic-major walk.  Dense meshes on hub rows exercise the Dhi prune ranks,
    opportunistic grafting every other tick the median; churn and fanout
    publishers outside their topics included.  Bit-exact against the oracle
    every tick."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from tickrun import restrict_to_subscriptions, run_parity, subscribed_schedule
    rng = np.random.default_rng(909)
    n, T = 3000, 8
    net = graphs.power_law(n, 16, 2.5, 1024, seed=41, n_topics=T)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 3, seed=42))
    deg = np.diff(net.row_ptr.astype(np.int64))
    assert deg.max() > 256 and ((deg > 64) & (deg <= 256)).sum() > 10, "both hub classes present"
    params = beacon_params(T, RetainScore=3 * Second)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300,
                             OpportunisticGraftThreshold=5)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second, OpportunisticGraftTicks=2)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.3)
    restrict_to_subscriptions(st, net)
    ticks = list(range(1, 7))
    sched = subscribed_schedule(rng, ticks, net, T, 2.0, 0.02, member_only=False)
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 50, replace=False)]
    churn = {3: [(down, False)], 5: [(down, True)]}
    run_parity(net, params, th, gp, st, ticks, sched, ring=1024, churn=churn, topic_slots=topic_slots)


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("topic_slots,shards", [(0, 0), (24, 0), (0, 3), (24, 3), (0, 8), (24, 8)])
def test_c5_combined_wide_hubs_zipf_churn_px_verdicts(require_gpu, topic_slots, shards):
    """C5's whole shape on one engine and on 3 shards: a plain Chung-Lu
    power law (exponent 2.5, i0 = 1) whose hubs exceed 1024 connections (up
    to the 4096 cap: the heartbeat on 2 row positions per thread up to 2048 connections and 4
    beyond, PX on a block of 4 waves per hub observer),
    64 topics with Zipf subscriptions, dense meshes on the hubs (Dhi prune
    ranks over thousands of positions), churn, peer exchange with the
    connector, every validation verdict, fanout publishers outside their
    topics, and (topic_slots) per-topic sub-rings with member-compacted
    seen-set cells.  Bit-exact against the oracle every tick."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from tickrun import restrict_to_subscriptions, run_parity, subscribed_schedule
    rng = np.random.default_rng(3131)
    n, T = 20000, 64
    net = graphs.power_law(n, 16, 2.5, 4096, seed=31, n_topics=T, i0=1)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 8, seed=32))
    deg = np.diff(net.row_ptr.astype(np.int64))
    assert (deg > 1024).sum() >= 3 and deg.max() <= 4096, "hub rows above 1024 connections"
    params = beacon_params(T, RetainScore=3 * Second)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300,
                             AcceptPXThreshold=0.0, OpportunisticGraftThreshold=5)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second, OpportunisticGraftTicks=3,
                         PeerExchange=True)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.3)
    restrict_to_subscriptions(st, net)
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 0.6, 0.0, member_only=False,
                                verdicts=[0.9, 0.04, 0.03, 0.02, 0.01])
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 100, replace=False)]
    churn = {2: [(down, False)], 4: [(down, True)]}
    log = []
    eng = None
    if shards:
        from gsim.shard import ShardedEngine
        from tickrun import SEED
        eng = ShardedEngine(params, th, gossip=gp, shards=shards)
        eng.load_graph(net)
        eng.set_seed(SEED)
        st.push_to_engine(eng)
    run_parity(net, params, th, gp, st, ticks, sched, ring=2048, churn=churn, px_log=log, topic_slots=topic_slots,
               eng=eng)
    assert sum(log) > 0, "PX made connections"


@pytest.mark.gpu
@pytest.mark.parametrize("max_frontier", [256, 4096])
def test_list_overflow_fallbacks_bit_exact(require_gpu, max_frontier):
    """The round lists of member-compacted layouts sized far below a round's
    first deliveries (gsim_msg_config.max_frontier): the claim list overflows
    (the commit falls back to k_commit's word scan), the forwarder list
    overflows (its entries that fit become fresh bits, k_flist_fresh, and the
    send scans them, k_send_tm), and quiet rounds still fit both.  c5's shape
    (power law with hubs, Zipf topics on sub-rings, churn, every verdict);
    bit-exact against the oracle every tick (the c5 line ran on these
    fallbacks before its lists were sized to 4 N)."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from tickrun import restrict_to_subscriptions, run_parity, subscribed_schedule
    rng = np.random.default_rng(5150)
    n, T = 6000, 16
    net = graphs.power_law(n, 16, 2.5, 1024, seed=51, n_topics=T, i0=1)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 4, seed=52))
    params = beacon_params(T, RetainScore=3 * Second)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300,
                             OpportunisticGraftThreshold=5)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second, OpportunisticGraftTicks=3)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.3)
    restrict_to_subscriptions(st, net)
    ticks = list(range(1, 5))
    sched = subscribed_schedule(rng, ticks, net, T, 1.0, 0.0, member_only=False,
                                verdicts=[0.9, 0.04, 0.03, 0.02, 0.01])
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 100, replace=False)]
    churn = {2: [(down, False)], 3: [(down, True)]}
    run_parity(net, params, th, gp, st, ticks, sched, ring=T * 24, churn=churn, topic_slots=24,
               max_frontier=max_frontier)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_rows_over_4096_bit_exact(require_gpu):
    """Hub rows of 6000 and 5000 connections (the reference's heartbeat and
    ipColocationFactor have no degree bound, gossipsub.go:1386-1557,
    score.go:344-388): their heartbeat runs on a block of 1024 threads with 8
    row positions each and the group state in global scratch
    (k_heartbeat_hub_g), fanout maintenance and publication likewise, PX lists
    on the 8192-position k_px_emit, P6 in 4096-key tiles.  A power law with
    two such hubs, dense hub meshes (Dhi prunes over thousands of positions),
    opportunistic grafting, churn, PX, sybil IPs on the hubs, fanout
    publishers and every verdict; bit-exact against the oracle every tick."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from gsim.engine import Network
    from tickrun import restrict_to_subscriptions, run_parity, subscribed_schedule
    rng = np.random.default_rng(8192)
    n, T = 8000, 6
    base = graphs.power_law(n, 12, 2.5, 1024, seed=81, n_topics=T, i0=1)
    src = base.owner()
    u = [src[src < base.col].astype(np.int64)]
    v = [base.col[src < base.col].astype(np.int64)]
    for hub, deg in ((0, 6000), (1, 5000)):
        others = rng.choice(np.arange(2, n), size=deg, replace=False)
        u.append(np.full(deg, hub, np.int64))
        v.append(others.astype(np.int64))
    u, v = np.concatenate(u), np.concatenate(v)
    a_, b_ = np.minimum(u, v), np.maximum(u, v)
    key = np.unique(a_ * n + b_)
    a_, b_ = key // n, key % n
    flip = rng.random(len(a_)) < 0.5                    # who dialled
    row_ptr, col, outbound = graphs._csr_from_pairs(n, np.where(flip, b_, a_), np.where(flip, a_, b_))
    deg = np.diff(row_ptr.astype(np.int64))
    assert deg[0] >= 6000 and deg[1] >= 5000 and deg.max() <= 8192
    ip_ids = np.arange(n, dtype=np.uint32)
    ip_ids[2:2000] = 2 + (np.arange(1998) // 25)          # sybil IPs shared by 25 peers each
    net = Network(n, row_ptr, col, outbound, np.full(n, (1 << T) - 1, dtype=np.uint64),
                  np.arange(n + 1, dtype=np.uint32), ip_ids, int(ip_ids.max()) + 1)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 3, seed=82))
    sub = net.sub.copy()
    sub[:2] = (1 << T) - 1                                # the hubs hold every topic
    net = graphs.with_subscriptions(net, sub)
    params = beacon_params(T, RetainScore=3 * Second)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300,
                             AcceptPXThreshold=0.0, OpportunisticGraftThreshold=5)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second, OpportunisticGraftTicks=2,
                         PeerExchange=True)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.3)           # hub meshes far over Dhi: prunes over thousands
    restrict_to_subscriptions(st, net)
    ticks = list(range(1, 5))
    sched = subscribed_schedule(rng, ticks, net, T, 1.5, 0.0, member_only=False,
                                verdicts=[0.85, 0.05, 0.04, 0.03, 0.03])
    s2 = net.owner()
    und = np.stack([s2, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=len(und) // 80, replace=False)]
    churn = {2: [(down, False)], 4: [(down, True)]}
    log = []
    run_parity(net, params, th, gp, st, ticks, sched, ring=1024, churn=churn, px_log=log)
