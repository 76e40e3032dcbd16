#!/usr/bin/env python3
"""Round-by-round engine vs oracle comparison of the delivery path (debug aid)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
import numpy as np  # noqa: E402

import oracle_binding as ob  # noqa: E402
from fixtures import beacon_params, beacon_topic, synthetic_state  # noqa: E402
from gsim import _abi  # noqa: E402
from gsim.engine import Engine, random_regular  # noqa: E402
from gsim.params import GossipSubParams, PeerScoreThresholds, Second  # noqa: E402
from test_delivery import HB, R, T0, _schedule  # noqa: E402
from test_heartbeat import SEED, tick_time  # noqa: E402

CASES = {
    "a": (1500, 16, 2, [1, 2, 3, 4], 6, 0.1, 0.0, 64),
    "b": (3000, 32, 3, [14, 15, 16], 12, 0.05, 0.03, 64),
}
n, k, T, ticks, rate, inv_frac, retained, ring = CASES[sys.argv[1] if len(sys.argv) > 1 else "a"]
rng = np.random.default_rng(n + k)
params = beacon_params(T)
params.Topics["topic01"] = beacon_topic(MeshMessageDeliveriesWindow=150 * 10**6)
gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
th = PeerScoreThresholds(GossipThreshold=-100, PublishThreshold=-200, GraylistThreshold=-300)
net = random_regular(n, k, seed=n, n_topics=T)
st = ob.NetState(net, params, thresholds=th, gossip=gp)
synthetic_state(st, rng, tick_time(0), 8 / k)
r = rng.random(net.e)
st.estate[r < retained] = _abi.ES_TRACKED
st.expire[r < retained] = tick_time(0) + rng.integers(1, 5, int((r < retained).sum())) * Second
st.bp[rng.random(net.e) < 0.02] = 40.0
msgs = ob.Msgs(n, T, ring, R, T0, HB)
eng = Engine(params, th, gossip=gp)
eng.load_graph(net)
eng.set_seed(SEED)
st.push_to_engine(eng)
eng.msgs_init(ring, R, T0, HB)
sched = _schedule(rng, ticks, T, R, rate, inv_frac, n)
lib = ob.load()
owner = np.repeat(np.arange(n), np.diff(net.row_ptr.astype(np.int64)))


def cmp(tag):
    gpu = ob.NetState(net, params, thresholds=th, gossip=gp)
    gpu.pull_from_engine(eng)
    bad = []
    for f in st.TOPIC_FIELDS + st.EDGE_FIELDS + ("ctl",):
        a, b = getattr(st, f), getattr(gpu, f)
        av = a.view(np.uint64) if a.dtype.itemsize == 8 else a
        bv = b.view(np.uint64) if b.dtype.itemsize == 8 else b
        if not np.array_equal(av, bv):
            idx = np.argwhere(av != bv)
            bad.append((f, len(idx), [(tuple(int(x) for x in i), a[tuple(i)], b[tuple(i)]) for i in idx[:6]]))
    seen = eng.read(_abi.F_SEEN)
    if not np.array_equal(seen, msgs.seen):
        idx = np.argwhere(seen != msgs.seen)
        bad.append(("seen", len(idx), [(tuple(int(x) for x in i), msgs.seen[tuple(i)], seen[tuple(i)]) for i in idx[:6]]))
    st_g = eng.msg_stats()
    if st_g != msgs.stats:
        bad.append(("stats", msgs.stats, st_g))
    if bad:
        print("MISMATCH after", tag)
        for b in bad:
            print("  ", b)
        for f, cnt, items in [b for b in bad if b[0] in ("first", "meshd", "invalid")]:
            for (t, e), c, g in items:
                print(f"    {f} t={t} e={e} receiver={owner[e]} sender={net.col[e]} score={st.score[e]} "
                      f"tflags={st.tflags[t, e]} estate={st.estate[e]}")
                for slot in range(ring):
                    if msgs.topic[slot] == t and msgs.seen[slot, owner[e]] != ob.UNSEEN:
                        print(f"      slot {slot} origin {msgs.origin[slot]} inv {msgs.invalid[slot]} "
                              f"seen(recv)={msgs.seen[slot, owner[e]]} seen(sender)={msgs.seen[slot, net.col[e]]} "
                              f"gpu seen(recv)={seen[slot, owner[e]]}")
        return True
    return False


for kk in ticks:
    now = tick_time(kk)
    eng.refresh_scores(now)
    v = st.view()
    lib.orc_refresh_scores(v, now)
    lib.orc_ip_colocation(v)
    lib.orc_compute_scores(v)
    if cmp(f"refresh {kk}"):
        sys.exit(1)
    eng.heartbeat(kk, now)
    lib.orc_heartbeat(v, kk, now, SEED)
    if cmp(f"heartbeat {kk}"):
        sys.exit(1)
    for g in range(kk * R, kk * R + R):
        for (mid, t, o, inv) in sched.get(g, []):
            msgs.publish(st, mid, t, o, inv, g)
        if g in sched:
            eng.publish(sched[g], g)
            pass
        msgs.round(st, g)
        eng.round(g)
        if cmp(f"round {g}"):
            sys.exit(1)
print("all rounds identical", msgs.stats)
