import sys, os
sys.path.insert(0, "go-libp2p-pubsub_amd"); sys.path.insert(0, "tests")
import numpy as np
import oracle_binding as ob
from fixtures import beacon_params, synthetic_state
from gsim.engine import random_regular
from gsim import wire
from gsim.params import GossipSubParams, PeerScoreThresholds, Second
from test_heartbeat import tick_time
from tickrun import run_parity, subscribed_schedule
import gsim.wire as W
n, k, T = 400, 16, 2
names = [f"t{t}".encode() for t in range(T)]
th = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-100, GraylistThreshold=-300)
params = beacon_params(T)
for case in ("window", "px"):
    rng = np.random.default_rng(7)
    if case == "window":
        gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2, MaxIHaveLength=2); rate, p_mesh = 8.0, 6 / k
    else:
        gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2, PeerExchange=True); rate, p_mesh = 2.0, 14 / k
    net = random_regular(n, k, seed=33, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), p_mesh)
    ticks = [1, 2, 3]
    sched = subscribed_schedule(rng, ticks, net, T, rate, 0.0)
    print(case, "sched", {g: len(v) for g, v in sched.items()} if isinstance(sched, dict) else type(sched))
    def ah(kk, eng, st_, msgs):
        try:
            r = wire.heartbeat_rpcs(eng, kk, 0, n, names, prune_backoff_s=60)
            print(case, kk, "no error:", len(r), "rpcs", sum(len(x[2]) for x in r), "bytes")
            print("ctl px bits", int(((st_.ctl[0] & 4) != 0).sum()), "prunes", int(((st_.ctl[0] & 2) != 0).sum()))
        except W.WireError as e:
            print(case, kk, "error:", e)
    run_parity(net, params, th, gp, st, ticks, sched, ring=256, after_heartbeat=ah)
