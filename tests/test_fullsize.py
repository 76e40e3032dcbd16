"""Parity at the benchmarked sizes (VERDICT r5 "Next" #2): the bench's own
networks, built by bench.py exactly as its line is measured (graph, the
device fill gsim_fill_synthetic, seeds, message schedule, adversaries), run
through gsim_step and compared with the oracle plane by plane.

* C3 at 1M peers x 16 topics (5.12e8 records): one full tick.  The oracle
  takes about a minute on 16 host threads (profiles/cpu_full_c3_box16.json)
  and the state about 40 GB of host memory.
* C4 at 125k peers (20 % sybils, 50 per IP, ignoring IWANT, opportunistic
  grafting every 10 heartbeats): ticks 1-10, across the opportunistic-graft
  tick, compared after every tick.

They take minutes, so they run only with GSIM_FULL_SIZE=1 (tools/gpu_r06_fullsize.sh
runs them with -s: each phase prints a progress line)."""
import os
import sys
import time

import numpy as np
import pytest

import oracle_binding as ob
from conftest import REPO
from gsim import _abi

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.environ.get("GSIM_FULL_SIZE"),
                                 reason="full-size parity: GSIM_FULL_SIZE=1 (minutes, ~40 GB host memory)")]


def _say(msg):
    print(f"[fullsize {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def _compare(st, eng, msgs, kk):
    """Totals, seen-set, mcache puts, then every state plane one field at a
    time (host memory stays bounded at the bench's size)."""
    assert eng.msg_stats() == msgs.stats, f"totals differ at tick {kk}: {eng.msg_stats()} vs {msgs.stats}"
    assert np.array_equal(eng.read(_abi.F_SEEN), msgs.seen), f"seen-set differs at tick {kk}"
    assert np.array_equal(eng.read(_abi.F_LASTPUT), msgs.lastput), f"mcache puts differ at tick {kk}"
    fields = [(f, st.FIELD_IDS[f]) for f in st.TOPIC_FIELDS + st.EDGE_FIELDS]
    fields += [("ctl", _abi.F_CTL), ("lastpub", _abi.F_LASTPUB), ("fan_topics", _abi.F_FANOUT_TOPICS)]
    for name, fid in fields:
        a = getattr(st, name)
        b = eng.read(fid)
        av = a.view(np.uint64) if a.dtype.itemsize == 8 else a
        bv = b.view(np.uint64) if b.dtype.itemsize == 8 else b
        if not np.array_equal(av, bv):
            bad = np.argwhere(av != bv)
            idx = tuple(bad[0])
            raise AssertionError(f"{name} differs at tick {kk}: {len(bad)} mismatches, first {idx}: "
                                 f"oracle={a[idx]!r} engine={b[idx]!r}")
        del b


def _bench_parity(config, ticks):
    sys.path.insert(0, REPO)
    import bench
    import gsim
    from gsim.presets import beacon_params, beacon_thresholds
    cfg = bench.CONFIGS[config]
    scen = bench.SCENARIOS.get(config, {})
    n, k, T, D, Dlo, Dhi = cfg
    seed = 1
    _say(f"{config}: building the bench network ({n} peers, k={k}, {T} topics) and its device fill")
    eng, net = bench.build_engine(cfg, seed, 0, scen)
    _, beh = bench.build_network(cfg, seed, scen)
    params = beacon_params(T)
    gp = gsim.GossipSubParams(D=D, Dlo=Dlo, Dhi=Dhi)
    if "opp_ticks" in scen:
        gp.OpportunisticGraftTicks = scen["opp_ticks"]
    st = ob.NetState(net, params, thresholds=beacon_thresholds(), gossip=gp)
    st.pull_from_engine(eng)                       # the oracle starts from the engine's fill
    _say(f"{config}: state pulled ({net.e} edges x {T} topics)")
    msgs = ob.Msgs(n, T, bench.MSG_RING, bench.ROUNDS, bench.tick_time(0), bench.SECOND, behaviour=beh)
    sched = bench.message_schedule(n, T, range(1, max(ticks) + 1))
    lib = ob.load()
    lib.orc_set_threads(int(os.environ.get("OMP_NUM_THREADS", min(16, os.cpu_count() or 1))))
    hb_seed = 0x5EED0000 + seed                    # build_engine's gsim_set_seed
    v = st.view()
    R = bench.ROUNDS
    for kk in ticks:
        now = bench.tick_time(kk)
        eng.step(kk, 1, {g: sched[g] for g in range(kk * R, kk * R + R) if g in sched})
        eng.synchronize()
        _say(f"{config}: engine tick {kk} done; oracle tick {kk} ...")
        lib.orc_refresh_scores(v, now)
        msgs.penalties(st, now)
        lib.orc_ip_colocation(v)
        lib.orc_compute_scores(v)
        msgs.heartbeat(st, kk, now, hb_seed)
        _say(f"{config}: oracle heartbeat {kk} done")
        for g in range(kk * R, kk * R + R):
            for m in sched.get(g, []):
                msgs.publish(st, int(m["id"]), int(m["topic"]), int(m["origin"]), int(m["verdict"]), g)
            msgs.round(st, g)
        _say(f"{config}: oracle rounds of tick {kk} done; comparing")
        _compare(st, eng, msgs, kk)
        _say(f"{config}: tick {kk} bit-exact ({msgs.stats[0]} deliveries so far)")
    eng.close()
    return msgs.stats


def test_c3_full_size_one_tick_bit_exact(require_gpu):
    """The bench's C3 line network (1M peers, k = 32, 16 topics, beacon
    params, 4 msg/s/topic): one tick through gsim_step against the oracle,
    every plane of the 5.12e8 records, the 1024 x 1M seen-set and the totals."""
    stats = _bench_parity("c3", [1])
    assert stats[0] > 10 ** 8, "a full tick of deliveries"


def test_c4_full_size_bit_exact(require_gpu):
    """The bench's C4 network (125k peers, 20 % sybils 50 per IP ignoring
    IWANT, opportunistic grafting every 10 heartbeats): ticks 1-10 against the
    oracle, tick 10 being an opportunistic-graft tick; the P6 counts of the
    sybils' shared IPs are in the compared score planes."""
    stats = _bench_parity("c4", list(range(1, 11)))
    assert stats[0] > 0
