"""Graph-sharded networks on the GPU: one
network split over 2-4 shards held in this process on one MI355X, exchanging
message copies, GRAFT/PRUNE records, gossip marks and IHAVE holders through
the in-process transport (the same group code the RCCL transport drives
across GPUs).  Every array of the whole network, assembled from the shards'
owned parts, is compared bit-for-bit with the single-network oracle after
every tick."""
import numpy as np
import pytest

import oracle_binding as ob
from gsim import _abi
from gsim.params import GossipSubParams, PeerScoreThresholds, Second

from test_heartbeat import tick_time


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("shards", [2, 4, 8])
def test_sharded_c3_shape_bit_exact(require_gpu, shards):
    """C3's shape (random-regular k=32, 16 topics, beacon-style params and
    thresholds) at 20k peers from the device fill, 5 ticks at 4 msg/s/topic
    with 2 % invalid messages: mesh maintenance, control, gossip, promises."""
    from fixtures import beacon_params, beacon_thresholds
    from gsim.engine import random_regular
    from gsim.shard import ShardedEngine
    from tickrun import SEED, run_parity, subscribed_schedule
    rng = np.random.default_rng(909 + shards)
    n, T = 20_000, 16
    net = random_regular(n, 32, seed=23, n_topics=T)
    params = beacon_params(T)
    th = beacon_thresholds()
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12)
    eng = ShardedEngine(params, th, gossip=gp, shards=shards)
    eng.load_graph(net)
    eng.set_seed(SEED)
    eng.fill_synthetic(seed=37, now=tick_time(0), p_mesh=8 / 32)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    st.pull_from_engine(eng)
    assert (st.tflags & _abi.TF_MESH).any() and (st.first != 0).any()
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.02)
    msgs, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=1024, eng=eng)
    assert gs["iwant_ids"] > 0 and gs["iwant_responses"] > 0
    assert msgs.stats[0] == msgs.stats[1] + msgs.stats[2]


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("cap,verdicts", [(64, None), (1024, (0.85, 0.05, 0.04, 0.03, 0.03))])
def test_sharded_power_law_churn_fanout_sybils(require_gpu, cap, verdicts):
    """A power-law graph (rows 1-64, or with hub rows up to ~500) over 3
    shards with Zipf subscriptions, publishers outside their topic (fanout),
    sybils sharing IPs that ignore IWANT (broken promises), direct peers,
    retained peers, connections churning between ticks (and every validation
    verdict with the hubs)."""
    from fixtures import beacon_params, synthetic_state
    from gsim import graphs
    from gsim.shard import ShardedEngine
    from tickrun import SEED, restrict_to_subscriptions, run_parity, subscribed_schedule
    rng = np.random.default_rng(4242)
    n, T = 4000, 12
    net = graphs.power_law(n, 16, 2.5, cap, seed=31, n_topics=T)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 4, seed=32))
    ip_ptr, ip_ids, n_ips, syb = graphs.sybil_ips(n, 0.1, 40, seed=33)
    net = graphs.with_ips(net, ip_ptr, ip_ids, n_ips)
    params = beacon_params(T, RetainScore=3 * Second)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.3)
    restrict_to_subscriptions(st, net)
    r = rng.random(net.e)
    st.estate[r < 0.02] = _abi.ES_TRACKED                       # retained peers
    st.expire[r < 0.02] = tick_time(0) + 2 * Second
    st.direct[:] = (rng.random(net.e) < 0.01).astype(np.uint8)
    st.direct[:] = st.direct | st.direct[st.rev]                # WithDirectPeers is mutual here
    beh = syb.astype(np.uint8) * ob.ORC_BEHAVE_IGNORE_IWANT
    eng = ShardedEngine(params, th, gossip=gp, shards=3)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st.push_to_engine(eng)
    ticks = list(range(1, 7))
    sched = subscribed_schedule(rng, ticks, net, T, 2.0, 0.03, member_only=False, verdicts=verdicts)
    src = net.owner()
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    downs = {k: und[rng.choice(len(und), size=len(und) // 40, replace=False)] for k in (2, 4)}
    churn = {2: [(downs[2], False)], 4: [(downs[2], True), (downs[4], False)], 6: [(downs[4], True)]}
    _, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=1024, behaviour=beh, churn=churn, eng=eng)
    assert gs["broken_promises"] > 0 and gs["iwant_ids"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rccl_single_rank_group_bit_exact(require_gpu):
    """The RCCL transport end to end on the one GPU a test box has: a
    one-rank communicator (gsim_group_create_rccl; counts by ncclAllGather,
    totals by ncclAllReduce) running a gossip network bit-exact against the
    oracle.  The exchange logic above the transport is the in-process tests'
    (RCCL refuses two ranks on one device, so K > 1 over RCCL runs only in
    the multi-GPU bench)."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from gsim.shard import ShardedEngine
    from tickrun import SEED, run_parity, subscribed_schedule
    rng = np.random.default_rng(77)
    n, T = 3000, 4
    net = random_regular(n, 16, seed=5, n_topics=T)
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    uid = ShardedEngine.rccl_unique_id()
    eng = ShardedEngine(params, th, gossip=gp, shards=1, rccl=(0, uid, 0))
    eng.load_graph(net)
    eng.set_seed(SEED)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.5)
    st.push_to_engine(eng)
    ticks = list(range(1, 5))
    sched = subscribed_schedule(rng, ticks, net, T, 4.0, 0.03)
    msgs, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=512, eng=eng)
    assert msgs.stats[1] > n and gs["iwant_ids"] >= 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_sharded_gossip_truncation_and_retransmission(require_gpu):
    """3 shards with MaxIHaveLength below the topics' gossip windows (the
    per-peer IHAVE subsets and the IWANT cap, k_ihave_pairs on ghost
    advertisers) and bad-signature messages served at most
    GossipRetransmission times per (message, peer)."""
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    from gsim.shard import ShardedEngine
    from tickrun import SEED, run_parity, subscribed_schedule
    rng = np.random.default_rng(515)
    n, T = 2400, 6
    net = random_regular(n, 16, seed=41, n_topics=T)
    params = beacon_params(T)
    th = PeerScoreThresholds(GossipThreshold=-20000, PublishThreshold=-50000, GraylistThreshold=-80000)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, MaxIHaveLength=6, GossipRetransmission=1)
    eng = ShardedEngine(params, th, gossip=gp, shards=3)
    eng.load_graph(net)
    eng.set_seed(SEED)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 0.5)
    st.push_to_engine(eng)
    ticks = list(range(1, 6))
    sched = subscribed_schedule(rng, ticks, net, T, 8.0, 0.0, verdicts=(0.7, 0.05, 0.05, 0.0, 0.2))
    _, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=1024, eng=eng)
    assert gs["iwant_ids"] > 0 and gs["iwant_responses"] > 0
