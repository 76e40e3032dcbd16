"""One shard per process: two processes on the test box's one
GPU, each hosting one shard of the network through gsim_group_create_host,
whose exchanges go device -> pinned host -> gloo all-to-all(v) / all-reduce
-> device.  That is the code path of the RCCL transport — one local shard,
per-rank counts, payloads by all-to-all(v), totals by all-reduce — with a
transport that runs two ranks on one device (RCCL refuses that).  Each rank
runs the oracle over the whole network and compares the state, seen-set and
mcache puts its shard owns, and the group totals, after every tick: copies
pushed to the other shard, control records, router state, gossip marks and
IHAVE holders all cross the process boundary."""
import os
import socket
import traceback

import numpy as np
import pytest


def _rank_main(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        from datetime import timedelta

        import torch.distributed as dist
        # a rank that fails leaves the other blocked in a collective: time out
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
        import oracle_binding as ob
        from fixtures import beacon_params, synthetic_state
        from gsim import _abi, graphs
        from gsim.params import GossipSubParams, PeerScoreThresholds, Second
        from gsim.shard import HostCollectives, ShardedEngine
        from test_heartbeat import tick_time
        from tickrun import SEED, restrict_to_subscriptions, run_parity, subscribed_schedule
        rng = np.random.default_rng(2718)
        n, T = 3000, 6
        net = graphs.power_law(n, 14, 2.5, 200, seed=41, n_topics=T)
        net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, 3, seed=42))
        params = beacon_params(T)
        th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
        gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2, FanoutTTL=3 * Second)
        st = ob.NetState(net, params, thresholds=th, gossip=gp)
        synthetic_state(st, rng, tick_time(0), 0.35)
        restrict_to_subscriptions(st, net)
        coll = HostCollectives()
        eng = ShardedEngine(params, th, gossip=gp, shards=world, host=(rank, coll, 0))
        eng.load_graph(net)
        eng.set_seed(SEED)
        st.push_to_engine(eng)
        ticks = list(range(1, 6))
        sched = subscribed_schedule(rng, ticks, net, T, 3.0, 0.03, member_only=False)
        src = net.owner()
        und = np.stack([src, net.col], axis=1)
        und = und[und[:, 0] < und[:, 1]]
        down = und[rng.choice(len(und), size=len(und) // 50, replace=False)]
        churn = {2: [(down, False)], 4: [(down, True)]}
        msgs, gs = run_parity(net, params, th, gp, st, ticks, sched, ring=1024, churn=churn, eng=eng,
                              local_only=True)
        q.put((rank, [int(x) for x in msgs.stats], gs, None))
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent
        q.put((rank, None, None, traceback.format_exc() + str(ex)))


def _diverge_main(rank, world, port, q):
    """The ranks' control flow diverges on purpose: rank 0 runs a heartbeat
    (its control exchange), rank 1 a tick's first round (its frontier
    exchange).  Both count exchanges are K x 8 B, so the transport itself
    sees nothing wrong; the tags must (gsim error ESTATE on both ranks,
    before any payload: no gloo abort, no hang)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        from datetime import timedelta

        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
        import oracle_binding as ob
        from fixtures import beacon_params, synthetic_state
        from gsim import _abi
        from gsim.engine import GsimError, random_regular
        from gsim.params import GossipSubParams, PeerScoreThresholds, Second
        from gsim.shard import HostCollectives, ShardedEngine
        from test_delivery import R, T0
        from test_heartbeat import tick_time
        from tickrun import SEED
        n, T = 600, 2
        net = random_regular(n, 12, seed=3, n_topics=T)
        params = beacon_params(T)
        th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-40, GraylistThreshold=-300)
        gp = GossipSubParams(D=6, Dlo=5, Dhi=10)
        st = ob.NetState(net, params, thresholds=th, gossip=gp)
        synthetic_state(st, np.random.default_rng(5), tick_time(0), 0.5)
        eng = ShardedEngine(params, th, gossip=gp, shards=world, host=(rank, HostCollectives(), 0))
        eng.load_graph(net)
        eng.set_seed(SEED)
        st.push_to_engine(eng)
        eng.msgs_init(64, R, T0, Second)
        eng.refresh_scores(tick_time(1))
        err, rc = None, None
        try:
            if rank == 0:
                eng.heartbeat(1, tick_time(1))
            else:
                eng.round(1 * R)
        except GsimError as ex:
            err, rc = str(ex), ex.rc
        assert err is not None and "exchange sequence mismatch" in err and rc == _abi.GSIM_ESTATE, err
        q.put((rank, err, None, None))
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent
        q.put((rank, None, None, traceback.format_exc() + str(ex)))


def _spawn(target, world=2):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    return q, [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_diverged_exchange_sequence_is_an_error_not_an_abort(require_gpu):
    q, procs = _spawn(_diverge_main)
    for pr in procs:
        pr.start()
    res = []
    try:
        for _ in procs:
            r = q.get(timeout=240)
            assert r[3] is None, f"rank {r[0]}: {r[3]}"
            res.append(r)
    finally:
        for pr in procs:
            pr.join(timeout=30)
            if pr.is_alive():
                pr.kill()
    assert sorted(r[0] for r in res) == [0, 1]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_two_processes_one_shard_each_bit_exact(require_gpu):
    q, procs = _spawn(_rank_main)
    for pr in procs:
        pr.start()
    import queue
    import time
    res = []
    try:
        t_end = time.time() + 540
        while len(res) < len(procs) and time.time() < t_end:
            try:
                r = q.get(timeout=5)
            except queue.Empty:
                if all(not pr.is_alive() for pr in procs):
                    break
                continue
            res.append(r)
            assert r[3] is None, f"rank {r[0]}: {r[3]}"        # the first failure ends the test
    finally:
        for pr in procs:
            pr.join(timeout=5 if len(res) < len(procs) else 60)
            if pr.is_alive():
                pr.kill()
    assert len(res) == len(procs), f"ranks reported: {[r[0] for r in res]}"
    (_, s0, g0, _), (_, s1, g1, _) = res
    assert s0 == s1 and s0[1] > 3000, s0
    assert g0 == g1 and g0["iwant_ids"] > 0, g0
