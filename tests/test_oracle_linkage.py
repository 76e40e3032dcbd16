"""The pin of the oracle's single-router structures carries over to the
network oracle that checks the GPU.

tests/test_oracle_kats.py pins `orc_mcache_*` (mcache_test.go),
`orc_gtracer_*` (gossip_tracer_test.go) and `orc_tcache_*` (timecache tests)
against the reference's own known answers.  The network oracle that runs
beside the engine (oracle_deliver.c / oracle_gossip.c) does not call them: it
derives every router's MessageCache windows from first-seen cells, its seen
cache from the dense seen array and its gossip tracer from a promise list.

This test runs the network oracle with its event log on (orc_msgs_log) over a
small network with gossip, IWANT-ignoring peers and mesh-isolated receivers,
then drives one pinned mcache, seen cache and gossip tracer per simulated
router with the logged events, and asserts per tick that both agree on:
  * GetGossipIDs(topic) of every router at every heartbeat (mcache.go:82-92);
  * the GetForPeer count of every IWANT served (mcache.go:66-80);
  * the seen verdict of every copy and publication (timecache Add);
  * GetBrokenPromises of every router at every penalty pass
    (gossip_tracer.go:79-115), after the same AddPromise / fulfill stream.
"""
import ctypes

import numpy as np

import oracle_binding as ob
from gsim.params import GossipSubParams, Second
from test_delivery import R, T0
from test_gossip import TH, cut_mesh, run_tick
from test_heartbeat import tick_time


def _network_run():
    from fixtures import beacon_params, synthetic_state
    from gsim.engine import random_regular
    n, k, T = 160, 10, 2
    rng = np.random.default_rng(71)
    net = random_regular(n, k, seed=17, n_topics=T)
    gp = GossipSubParams(D=6, Dlo=5, Dhi=12)
    st = ob.NetState(net, beacon_params(T), thresholds=TH, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 6 / k)
    beh = (rng.random(n) < 0.5).astype(np.uint8) * ob.ORC_BEHAVE_IGNORE_IWANT
    msgs = ob.Msgs(n, T, 128, R, T0, Second, behaviour=beh)
    msgs.log()
    mid = 0
    isolated = rng.choice(n, size=12, replace=False)
    for kk in range(1, 11):
        sched = {}
        for r in (1, 4, 7):
            batch = []
            for t in range(T):
                batch.append((mid, t, int(rng.integers(0, n)), 0))
                mid += 1
            sched[kk * R + r] = batch
        # some receivers outside every mesh this tick: they recover by IHAVE/IWANT
        cut = isolated[(kk % 3) * 4:(kk % 3) * 4 + 4]
        run_tick(st, msgs, kk, sched=sched, isolate=lambda: [cut_mesh(net, st, int(p)) for p in cut])
    return net, gp, msgs, msgs.events()


def test_network_oracle_matches_pinned_structures():
    net, gp, msgs, ev = _network_run()
    lib = ob.load()
    n = net.n
    mc = [lib.orc_mcache_new(gp.HistoryGossip, gp.HistoryLength) for _ in range(n)]
    tc = [lib.orc_tcache_new(0, 120 * Second) for _ in range(n)]
    gt = [lib.orc_gtracer_new(gp.IWantFollowupTime) for _ in range(n)]
    kinds = ev["kind"]
    seen = {k: 0 for k in range(1, 22)}
    buf = (ctypes.c_uint64 * 256)()
    peers = (ctypes.c_uint32 * 256)()
    counts = (ctypes.c_int32 * 256)()
    try:
        q = 0
        while q < len(ev):
            e = ev[q]
            kind = int(e["kind"])
            seen[kind] += 1
            a, b, mid, x = int(e["a"]), int(e["b"]), int(e["mid"]), int(e["x"])
            if kind == ob.EV_HEARTBEAT:
                # GetGossipIDs of every router and topic, then Shift
                want = {}
                q += 1
                while q < len(ev) and kinds[q] == ob.EV_GOSSIP_ID:
                    g = ev[q]
                    want.setdefault((int(g["a"]), int(g["topic"])), set()).add(int(g["mid"]))
                    seen[ob.EV_GOSSIP_ID] += 1
                    q += 1
                for p in range(n):
                    for t in range(2):
                        k = lib.orc_mcache_gossip_ids(mc[p], t, buf, 256)
                        got = set(buf[i] for i in range(k))
                        assert got == want.get((p, t), set()), f"tick {x}: GetGossipIDs({t}) of router {p}"
                for p in range(n):
                    lib.orc_mcache_shift(mc[p])
                continue
            if kind == ob.EV_PENALTIES:
                broken = {}
                q += 1
                while q < len(ev) and kinds[q] == ob.EV_BROKEN:
                    g = ev[q]
                    broken[(int(g["a"]), int(g["b"]))] = int(g["x"])
                    seen[ob.EV_BROKEN] += 1
                    q += 1
                got = {}
                for p in range(n):
                    k = lib.orc_gtracer_broken(gt[p], x, peers, counts, 256)
                    for i in range(k):
                        got[(p, int(peers[i]))] = int(counts[i])
                assert got == broken, f"broken promises at {x}"
                continue
            if kind == ob.EV_PUT:
                lib.orc_mcache_put(mc[a], mid, int(e["topic"]))
            elif kind == ob.EV_SEEN:
                assert lib.orc_tcache_add(tc[a], mid, msgs.round_time(int(e["g"]))) == x, \
                    f"seen verdict of {mid} at router {a}"
            elif kind == ob.EV_SERVE:
                cnt = ctypes.c_int32()
                assert lib.orc_mcache_get_for_peer(mc[a], mid, b, ctypes.byref(cnt)) == 1, "served from the cache"
                assert cnt.value == x, f"GetForPeer count of {mid} for {b} at router {a}"
            elif kind == ob.EV_PROMISE:
                m = ctypes.c_uint64(mid)
                lib.orc_gtracer_add_promise(gt[a], b, ctypes.byref(m), 1, 0, x)
            elif kind == ob.EV_FULFILL:
                lib.orc_gtracer_fulfill(gt[a], mid)
            q += 1
    finally:
        for p in range(n):
            lib.orc_mcache_free(mc[p])
            lib.orc_tcache_free(tc[p])
            lib.orc_gtracer_free(gt[p])
    # the stream exercised every structure
    assert seen[ob.EV_HEARTBEAT] == 10 and seen[ob.EV_GOSSIP_ID] > 0
    assert seen[ob.EV_SERVE] > 0 and seen[ob.EV_PROMISE] > 0 and seen[ob.EV_BROKEN] > 0
    assert seen[ob.EV_SEEN] > seen[ob.EV_PUT] > 0


def test_topic_subrings_assign_slots_in_publication_order():
    """gsim_msg_config.topic_slots: topic t's messages take slots
    t * topic_slots + (earlier messages of t mod topic_slots), whatever their
    ids; the seen-set rows of a slot start unseen except at the origin."""
    from fixtures import beacon_params
    from gsim.engine import random_regular
    n, T, R_t = 200, 3, 4
    net = random_regular(n, 8, seed=3, n_topics=T)
    st = ob.NetState(net, beacon_params(T), gossip=GossipSubParams(D=4, Dlo=3, Dhi=6))
    msgs = ob.Msgs(n, T, T * R_t, R, T0, Second, topic_slots=R_t)
    order = [(101, 1, 5), (7, 1, 9), (55, 0, 11), (3, 2, 13), (8, 1, 17), (9, 1, 19), (10, 1, 21)]
    for g, (mid, t, o) in enumerate(order):
        msgs.publish(st, mid, t, o, 0, g)
    # topic 1 took 1*4+0, +1, +2, +3, then wrapped to 1*4+0
    assert list(msgs.mid[4:8]) == [10, 7, 8, 9]
    assert msgs.mid[0] == 55 and msgs.mid[8] == 3
    assert list(msgs.topic) == [0] * 4 + [1] * 4 + [2] * 4
    assert msgs.seen[4, 21] == 6 and (msgs.seen[4] != ob.UNSEEN).sum() == 1
