#!/usr/bin/env python3
"""Run the oracle halves of the GPU parity tests that exercise churn and the
peer gater under AddressSanitizer + UBSan (a host-side
segfault in `orc_round` under test_churn_ticks_bit_exact).

The oracle sources are compiled to /tmp/orc_asan/liboracle.so with
`-fsanitize=address,undefined`, loaded through GSIM_ORACLE_LIB, and this
script re-executes itself with libasan preloaded (Python is not built with
ASan).  No GPU: only the oracle side of each test runs, with the tests' own
inputs.

usage: python tools/asan_oracle.py
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = "/tmp/orc_asan"


def build():
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(OUT, "liboracle.so")
    srcs = [os.path.join(REPO, "oracle", f) for f in
            ("oracle.c", "oracle_net.c", "oracle_deliver.c", "oracle_gossip.c", "oracle_gater.c")]
    subprocess.check_call(["gcc", "-O1", "-g", "-std=c11", "-fPIC", "-ffp-contract=off", "-fopenmp",
                           "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all",
                           "-shared", "-o", lib] + srcs + ["-lm"])
    return lib


def churn_case(n, k, T, nticks, rate, churn_frac):
    """tests/test_churn.py::test_churn_ticks_bit_exact, oracle side."""
    import numpy as np
    import oracle_binding as ob
    from fixtures import beacon_params, synthetic_state
    from gsim import _abi
    from gsim.engine import random_regular
    from gsim.params import GossipSubParams, PeerScoreThresholds, Second
    from test_delivery import R, T0, _schedule
    from test_heartbeat import SEED, tick_time
    rng = np.random.default_rng(n * 3 + k)
    params = beacon_params(T, RetainScore=3 * Second)
    gp = GossipSubParams(D=8, Dlo=6, Dhi=12, Dscore=4, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-20, PublishThreshold=-50, GraylistThreshold=-300)
    net = random_regular(n, k, seed=n + 7, n_topics=T)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 8 / k)
    st.bp[rng.random(net.e) < 0.05] = 12.0
    msgs = ob.Msgs(n, T, 256, R, T0, Second)
    sched = _schedule(rng, list(range(1, nticks + 1)), T, R, rate, 0.05, n)
    lib = ob.load()
    src = np.repeat(np.arange(n, dtype=np.uint32), np.diff(net.row_ptr).astype(np.int64))
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = []
    for kk in range(1, nticks + 1):
        now = tick_time(kk)
        if kk >= 2:
            if down:
                st.churn(down.pop(0), up=True, now=now - Second // 2)
            pick = und[rng.choice(len(und), size=max(1, int(churn_frac * len(und))), replace=False)]
            busy = {tuple(x) for batch in down for x in batch}
            pick = np.array([x for x in pick if tuple(x) not in busy], dtype=np.uint32)
            st.churn(pick, up=False, now=now - Second // 2)
            down.append(pick)
        v = st.view()
        lib.orc_refresh_scores(v, now)
        msgs.penalties(st, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
        msgs.heartbeat(st, kk, now, SEED)
        for g in range(kk * R, kk * R + R):
            for (mid, t, o, inv) in sched.get(g, []):
                msgs.publish(st, mid, t, o, inv, g)
            msgs.round(st, g)
    print("churn", (n, k, T), "stats", msgs.stats, "retained",
          int((((st.estate & _abi.ES_TRACKED) != 0) & ((st.estate & _abi.ES_CONNECTED) == 0)).sum()))


def gater_case(weights):
    """tests/test_gater.py::test_gater_network_bit_exact, oracle side."""
    import numpy as np
    import oracle_binding as ob
    from fixtures import beacon_params, sybil_ips, synthetic_state
    from gsim.engine import random_regular
    from gsim.params import GossipSubParams, PeerScoreThresholds, Second
    from gsim import NewPeerGaterParams
    from test_delivery import R, T0
    from test_heartbeat import SEED, tick_time
    from tickrun import subscribed_schedule
    n, k, T = 800, 16, 3
    rng = np.random.default_rng(404)
    net = random_regular(n, k, seed=77, n_topics=T)
    net.ip_ptr, net.ip_ids, net.n_ips = sybil_ips(n, 0.3, 6, rng)
    params = beacon_params(T)
    gp = GossipSubParams(D=6, Dlo=5, Dhi=10, Dscore=3, Dout=2)
    th = PeerScoreThresholds(GossipThreshold=-50, PublishThreshold=-100, GraylistThreshold=-400)
    st = ob.NetState(net, params, thresholds=th, gossip=gp)
    synthetic_state(st, rng, tick_time(0), 6 / k)
    ticks = list(range(1, 7))
    sched = subscribed_schedule(rng, ticks, net, T, 12.0, 0.0, verdicts=(0.45, 0.15, 0.1, 0.25, 0.05))
    src = np.repeat(np.arange(n, dtype=np.uint32), np.diff(net.row_ptr.astype(np.int64)))
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    down = und[rng.choice(len(und), size=40, replace=False)]
    churn = {3: [(down, False)], 5: [(down, True)]}
    gater = NewPeerGaterParams(0.05, 0.9, 0.99)
    if weights:
        gater.TopicDeliveryWeights = weights
    msgs = ob.Msgs(net.n, st.T, 512, R, T0, Second)
    st.enable_gater(gater)
    lib = ob.load()
    for kk in ticks:
        now = tick_time(kk)
        for (pairs, up) in churn.get(kk, []):
            st.churn(pairs, up=up, now=now - Second // 2)
        v = st.view()
        lib.orc_refresh_scores(v, now)
        st.gater_decay(now)
        msgs.penalties(st, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
        msgs.heartbeat(st, kk, now, SEED)
        for g in range(kk * R, kk * R + R):
            for msg in sched.get(g, []):
                msgs.publish(st, *msg[:4], g)
            msgs.round(st, g)
    print("gater", weights, "stats", msgs.stats, "throttled", st.gater_throttled())


def main():
    if os.environ.get("GSIM_ORACLE_LIB") is None:
        lib = build()
        asan = subprocess.check_output(["gcc", "-print-file-name=libasan.so"], text=True).strip()
        ubsan = subprocess.check_output(["gcc", "-print-file-name=libubsan.so"], text=True).strip()
        env = dict(os.environ, GSIM_ORACLE_LIB=lib, LD_PRELOAD=f"{asan}:{ubsan}",
                   ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
                   OMP_NUM_THREADS="1")
        sys.exit(subprocess.call([sys.executable, __file__] + sys.argv[1:], env=env))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
    churn_case(1200, 16, 2, 9, 8, 0.02)
    churn_case(2500, 32, 3, 8, 10, 0.05)
    gater_case(None)
    gater_case({0: 0.5, 2: 2.25})
    print("asan: clean")


if __name__ == "__main__":
    main()
