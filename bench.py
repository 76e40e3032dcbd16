#!/usr/bin/env python3
"""bench.py — peer-heartbeat updates/sec + msg-edge deliveries/sec on the
1M-peer, 16-topic network (C3), one MI355X per rank.

A "step" is one heartbeat tick of the whole simulated network with every byte
of state resident in HBM:
  refreshScores+score (decay, P1-P7 snapshot)        k_refresh_score
  heartbeat mesh maintenance (all peers, all topics)  k_heartbeat
  10 propagation rounds, each: publications (Poisson 4 msg/s/topic, seed 2),
  mesh forwarding + AcceptFrom + seen-set claims + duplicate/invalid
  counters, seen commit + first-delivery credit, control inbox (rounds 0-1)
                                                      k_publish, k_send,
                                                      k_commit, k_handle_control
W untimed warmup ticks, then exactly K timed ticks bracketed by barrier +
device sync; max over ranks; rank 0 prints one JSON line.  Per-kernel-class
device time comes from HIP events recorded on the engine stream around every
launch inside the timed region (gsim_profile).

Multi-GPU: the one network is graph-sharded over the ranks
(contiguous peer ranges, one shard per GPU), with the halo exchange of message
copies, GRAFT/PRUNE records, gossip marks and IHAVE holders over RCCL
(strong scaling: the same 1M-peer network at every N).  --replicas runs one
independent network per rank instead (weak scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

SECOND = 1_000_000_000
SALU_PEAK = 256 * 2.4e9       # scalar instructions/s: one scalar unit per CU
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# random 8-B load probes (tools/probe_random.hip, profiles/r01_probe_random_access.jsonl)
PROBE_MISS_PER_S = 54.1e9      # 2 GB table: every load an L2 miss
PROBE_L2_REQ_PER_S = 251.2e9   # 4 MB table: L2-resident
ROUNDS = 10                    # propagation rounds per heartbeat
MSG_RATE = 4.0                 # messages / s / topic
MSG_RING = 1024                # live-message window: >= 16 heartbeats of publications, so no slot
                               # is republished while its message can still be gossiped or promised
DUP_BYTES, FIRST_BYTES = 40, 72   # algorithmic bytes per delivery

CONFIGS = {
    # id: (peers, degree, topics, D, Dlo, Dhi)
    "c3": (1_000_000, 32, 16, 8, 6, 12),
    "c2": (10_000, 32, 1, 8, 6, 12),
    "c4": (125_000, 32, 1, 8, 6, 12),
    "c5": (10_000_000, 16, 64, 8, 6, 12),
}
# Structure beyond (peers, degree, topics, D) for the BASELINE configurations
# that are not plain random-regular networks:
#  c4  Sybil/eclipse: 100k honest + 25k sybils (20 %), one IP per 50 sybils
#      (P6), sybils ignore IWANT (broken promises -> P7), opportunistic
#      grafting every 10 heartbeats so the timed window holds it.
#  c5  10M peers, plain Chung-Lu power law (exponent 2.5, mean 16, i0 = 1:
#      hubs up to the 4096-connection cap), 64 topics with Zipf subscriptions
#      (8 per peer), 1 % of connections going down per tick and coming back
#      two ticks later, publishers are topic members, 4 msg/s/topic (256 msg/s
#      network-wide) over per-topic sub-rings of 128 slots (ring 8192, the
#      engine's maximum: ~32 ticks of publications per topic, so a slot is
#      reused only after its message has left every window -- 96 slots refused
#      runs past ~24 ticks), peer
#      exchange on (PRUNEs carry PX; the connector runs between ticks and
#      reconnects churned-down addresses).  Topic-slot planes and
#      member-compacted seen-set cells keep it in one GPU's
#      HBM (the dense layouts would need ~560 GB of planes and ~500 GB of
#      cells).
SCENARIOS = {
    "c4": {"sybil_frac": 0.2, "per_ip": 50, "opp_ticks": 10},
    "c5": {"power_law": (2.5, 4096), "i0": 1.0, "zipf_per_peer": 8, "churn_frac": 0.01, "topic_slots": 128,
           "msg_rate": 4.0, "px": True},
}


def _diag_phases(eng):
    """k_send_tm's phase clocks in a -DGSIM_DIAG_PHASE build (gsim_diag_send_phases, not part of
    gsim.h): resets them now and returns a reader of [all, scans + layouts, walks, waves, clocks
    of the later layers, chunk-layers, chunks, forwarders of the later layers]."""
    import ctypes
    fn = eng.lib.gsim_diag_send_phases
    fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    out = (ctypes.c_uint64 * 8)()
    fn(eng.h, out)

    def read():
        fn(eng.h, out)
        return list(out)
    return read


def host_syncs(eng) -> int:
    """The library's host synchronisations so far in this process (gsim_host_sync_count)."""
    import ctypes
    v = ctypes.c_uint64(0)
    eng.lib.gsim_host_sync_count(ctypes.byref(v))
    return int(v.value)


def box_info() -> dict:
    """The box a line was measured on (the same code measured 16 % apart on two
    boxes): host name and the GPU's current clock levels read from sysfs (pp_dpm_*: the level
    marked '*'), best effort.  No child process: under rocprofv3 every process the bench starts
    would initialise the GPU, and a launcher script's exec is refused on this pool."""
    import glob
    import socket
    out = {"host": socket.gethostname()}
    for clk in ("sclk", "mclk", "fclk"):           # one entry per DRM card the box shows
        vals = []
        for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
            try:
                with open(f"{dev}/pp_dpm_{clk}") as f:
                    cur = [ln.split(":", 1)[1].strip(" *\n") for ln in f if ln.rstrip().endswith("*")]
                if cur:
                    vals.append(cur[0])
            except OSError:
                pass
        if vals:
            out[clk] = vals
    return out


def _diag_hb(eng):
    """The heartbeat's counters in a -DGSIM_DIAG_HB build (gsim_diag_hb_counts, not part of
    gsim.h): resets them now and returns a reader of [re-scored positions, Grafts, Prunes,
    backoff loads]."""
    import ctypes
    fn = eng.lib.gsim_diag_hb_counts
    fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    out = (ctypes.c_uint64 * 4)()
    fn(eng.h, out)

    def read():
        fn(eng.h, out)
        return list(out)
    return read


def _diag_ih(eng):
    """The member-major IHAVE walk's counters in a -DGSIM_DIAG_IH build (gsim_diag_ih_counts,
    not part of gsim.h), per LP (1: rows of <= 256 connections, 2: the hub rows): push row
    walks, push edges, gossip targets among them, pull row walks, pull edges, gossiping
    advertisers among them, push and pull wave clocks.  Resets them now; returns a reader."""
    import ctypes
    fn = eng.lib.gsim_diag_ih_counts
    fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    out = (ctypes.c_uint64 * 16)()
    fn(eng.h, out)

    def read():
        fn(eng.h, out)
        names = ("push_walks", "push_edges", "push_targets", "pull_walks", "pull_edges", "pull_advertisers",
                 "push_clocks", "pull_clocks")
        return {f"lp{lp}": {k: int(out[8 * (lp - 1) + q]) for q, k in enumerate(names)} for lp in (1, 2)}
    return read


def refresh_bytes(census: dict, n_edges: int) -> int:
    """Compulsory HBM bytes of one refreshScores+score pass on this state
    (DESIGN.md §4.1): every connected scored record reads its 4 counters and
    flags (33 B); in-mesh records also read graftTime (8 B) -- with lazy
    meshTime the pass no longer stores meshTime; every
    non-zero counter changes under decay and is written (8 B); per edge:
    estate 1, bp r+w 16, P5 gather 8, col 4, P6 8, score write 8."""
    nz = census["nz_first"] + census["nz_meshd"] + census["nz_fail"] + census["nz_invalid"]
    return 33 * census["records"] + 8 * census["in_mesh"] + 8 * nz + 45 * n_edges


def tick_time(k: int) -> int:
    return 3600 * SECOND + k * SECOND


def message_schedule(n: int, T: int, ticks: range, seed: int = 2, sub=None, rate: float = MSG_RATE) -> dict:
    """{round: gsim_msg array}: Poisson(MSG_RATE) messages per topic per
    heartbeat, each in a uniform round of its tick, origin uniform (among
    the topic's members when `sub`, the subscription masks, is given)."""
    from gsim import _abi
    rng = np.random.default_rng(seed)
    members = None
    if sub is not None:
        members = [np.nonzero((sub >> np.uint64(t)) & np.uint64(1))[0] for t in range(T)]
    out, mid = {}, 0
    for k in ticks:
        per_round = [[] for _ in range(ROUNDS)]
        for t in range(T):
            for _ in range(rng.poisson(rate)):
                if members is not None and len(members[t]):
                    origin = int(members[t][rng.integers(0, len(members[t]))])
                else:
                    origin = int(rng.integers(0, n))
                per_round[int(rng.integers(0, ROUNDS))].append((mid, t, origin))
                mid += 1
        for r, lst in enumerate(per_round):
            if lst:
                a = np.zeros(len(lst), dtype=_abi.MSG_DTYPE)
                a["id"] = [x[0] for x in lst]
                a["topic"] = [x[1] for x in lst]
                a["origin"] = [x[2] for x in lst]
                out[k * ROUNDS + r] = a
    return out


def build_network(cfg, seed, scen=None):
    """The synthetic graph of a configuration; returns
    (network, per-peer behaviour flags or None)."""
    import gsim
    from gsim import _abi, graphs
    n, k, T = cfg[0], cfg[1], cfg[2]
    scen = scen or {}
    beh = None
    if "power_law" in scen:
        ex, cap = scen["power_law"]
        gen = graphs.power_law_native if n > 200_000 else graphs.power_law   # numpy: minutes at 10M
        net = gen(n, k, ex, cap, seed=seed, n_topics=T, i0=scen.get("i0"))
        net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(n, T, scen["zipf_per_peer"], seed=seed + 100))
    else:
        net = gsim.random_regular(n, k, seed=seed, n_topics=T)
    if "sybil_frac" in scen:
        ip_ptr, ip_ids, n_ips, syb = graphs.sybil_ips(n, scen["sybil_frac"], scen["per_ip"], seed=seed + 200)
        net = graphs.with_ips(net, ip_ptr, ip_ids, n_ips)
        beh = syb.astype(np.uint8) * np.uint8(_abi.BEHAVE_IGNORE_IWANT)
    elif not os.environ.get("GSIM_BENCH_NO_IPS"):   # (diagnostic A/B: the network without IP lists)
        # honest peers get a unique IP id (P6 is derived, and is 0)
        net = graphs.with_ips(net, np.arange(n + 1, dtype=np.uint32), np.arange(n, dtype=np.uint32), n)
    return net, beh


def build_engine(cfg, seed, device, scen=None, shard=None):
    """The bench network on one GPU, or (shard = (rank, world, unique_id))
    this rank's shard of it (gsim.shard.ShardedEngine over RCCL)."""
    import gsim
    from gsim.presets import beacon_params, beacon_thresholds
    n, k, T, D, Dlo, Dhi = cfg
    scen = scen or {}
    params = beacon_params(T)
    gp = gsim.GossipSubParams(D=D, Dlo=Dlo, Dhi=Dhi, PeerExchange=bool(scen.get("px")))
    if "opp_ticks" in scen:
        gp.OpportunisticGraftTicks = scen["opp_ticks"]
    if shard is None:
        eng = gsim.Engine(params, beacon_thresholds(), gossip=gp, device=device)
    elif isinstance(shard, int):          # every shard in this process, on this device
        from gsim.shard import ShardedEngine
        eng = ShardedEngine(params, beacon_thresholds(), gossip=gp, shards=shard, devices=[device] * shard)
    else:
        from gsim.shard import ShardedEngine
        rank, world, uid = shard
        eng = ShardedEngine(params, beacon_thresholds(), gossip=gp, shards=world, rccl=(rank, uid, device))
    net, beh = build_network(cfg, seed, scen)
    eng.load_graph(net)
    eng.set_seed(0x5EED0000 + seed)
    eng.fill_synthetic(seed=seed * 7919 + 1, now=tick_time(0), p_mesh=D / k)
    ts = scen.get("topic_slots", 0)
    eng.msgs_init(T * ts if ts else scen.get("ring", MSG_RING), ROUNDS, tick_time(0), SECOND,
                  max_arrivals=scen.get("max_arrivals"), topic_slots=ts)
    if beh is not None:
        eng.set_peer_behaviour(beh)
    if os.environ.get("GSIM_SEND_VARIANT") and shard is None:   # A/B of the delivery kernel (gsim.h)
        eng.set_kernel_variant(2, int(os.environ["GSIM_SEND_VARIANT"]))
    if os.environ.get("GSIM_TM_UNIFORM"):                        # topic-major blocks the same per topic
        eng.set_kernel_variant(6, int(os.environ["GSIM_TM_UNIFORM"]))
    if os.environ.get("GSIM_FLIST_OFF"):                         # sparse rounds by the fresh-bit scan (A/B)
        eng.set_kernel_variant(9, 1)
    if os.environ.get("GSIM_XB_GENERIC"):                        # the bit apply one copy at a time (A/B)
        eng.set_kernel_variant(8, 1)
    if os.environ.get("GSIM_IHAVE_W"):                           # the IHAVE walk's lane group (A/B)
        eng.set_kernel_variant(3, int(os.environ["GSIM_IHAVE_W"]))
    return eng, net


def describe_graph(cfg, scen) -> str:
    k = cfg[1]
    if "power_law" in scen:
        d = (f"Chung-Lu power law (exponent {scen['power_law'][0]:g}, mean {k}, rows <= {scen['power_law'][1]}"
             f"{', i0 = %g' % scen['i0'] if 'i0' in scen else ''}), "
             f"Zipf subscriptions ({scen['zipf_per_peer']} topics/peer)")
    else:
        d = f"random-regular k={k}"
    if "sybil_frac" not in scen:
        d += ", one IP per peer"
    if "sybil_frac" in scen:
        d += (f", {scen['sybil_frac']:.0%} sybils ({scen['per_ip']} per IP) ignoring IWANT, "
              f"opportunistic grafting every {scen['opp_ticks']} heartbeats")
    if "churn_frac" in scen:
        d += f", {scen['churn_frac']:.0%} of connections down per tick (back 2 ticks later)"
    if scen.get("px"):
        d += ", peer exchange"
    if scen.get("topic_slots"):
        d += f", per-topic sub-rings of {scen['topic_slots']} slots (member-compacted seen-set)"
    return d


def churn_schedule(net, frac: float, ticks: range, seed: int = 4) -> dict:
    """{tick: [(pairs, up)]}: a random `frac` of the undirected connections
    goes down before each tick and comes back two ticks later."""
    rng = np.random.default_rng(seed)
    src = np.repeat(np.arange(net.n, dtype=np.uint32), np.diff(net.row_ptr.astype(np.int64)))
    und = np.stack([src, net.col], axis=1)
    und = und[und[:, 0] < und[:, 1]]
    out, downs = {}, {}
    for k in ticks:
        ev = []
        if k - 2 in downs:
            ev.append((downs.pop(k - 2), True))
        downs[k] = und[rng.choice(len(und), size=max(1, int(len(und) * frac)), replace=False)]
        ev.append((downs[k], False))
        out[k] = ev
    return out


CALLTIME = None      # --calltime: wall ms per engine call (each one synchronised; diagnostic only)


def _timed(name, f, *a, **kw):
    if CALLTIME is None:
        return f(*a, **kw)
    t0 = time.perf_counter()
    r = f(*a, **kw)
    CALLTIME["_eng"].synchronize()
    CALLTIME[name] = CALLTIME.get(name, 0.0) + (time.perf_counter() - t0) * 1e3
    return r


def run_tick(eng, k, sched, churn=None, px=False):
    now = tick_time(k)
    for (pairs, up) in (churn or {}).get(k, []):
        _timed("set_connections", eng.set_connections, pairs, up=up, now=now - SECOND // 2)
    _timed("refresh_scores", eng.refresh_scores, now)
    _timed("heartbeat", eng.heartbeat, k, now)
    for g in range(k * ROUNDS, (k + 1) * ROUNDS):
        m = sched.get(g)
        if m is not None:
            _timed("publish", eng.publish_array, m, g)
        _timed("round", eng.round, g)
    if px:                                     # the connector for this tick's PX attempts
        _timed("px_connect", eng.px_connect, now + SECOND // 2, want_pairs=False)


def run_ticks(eng, k0, n, sched, churn=None, px=False):
    """Ticks k0+1 .. k0+n through gsim_step: one call for all of
    them when nothing happens between ticks, else one call per tick with the
    churn before and the PX connector after it.  --calltime, sharded groups
    and GSIM_BENCH_PHASES=1 use the per-phase calls (run_tick)."""
    if CALLTIME is not None or not hasattr(eng, "step") or os.environ.get("GSIM_BENCH_PHASES"):
        for kk in range(k0 + 1, k0 + n + 1):
            run_tick(eng, kk, sched, churn, px=px)
        return

    def part(a, b):
        return {g: sched[g] for g in range(a * ROUNDS, b * ROUNDS) if g in sched}

    if not churn and not px:
        eng.step(k0 + 1, n, part(k0 + 1, k0 + n + 1))
        return
    for kk in range(k0 + 1, k0 + n + 1):
        now = tick_time(kk)
        for (pairs, up) in (churn or {}).get(kk, []):
            eng.set_connections(pairs, up=up, now=now - SECOND // 2)
        eng.step(kk, 1, part(kk, kk + 1))
        if px:
            eng.px_connect(now + SECOND // 2, want_pairs=False)


def cpu_baseline(cfg, scen=None, n: int = 10_000, ticks: int = 5, budget_s: float = 25.0, warmup: int = 1,
                 legs=("single", "all")):
    """Time the C oracle on a bounded sample of the same workload (same graph
    model, degree, topics, parameters, adversaries, churn and message rate,
    `n` peers): one warm-up tick, then `ticks` ticks timed one by one, the
    median reported — once on one core and once with OpenMP over the host's
    threads in the parallel phases (refresh/score, heartbeat, control)."""
    import oracle_binding as ob
    from fixtures import beacon_params, beacon_thresholds, synthetic_state
    from tickrun import restrict_to_subscriptions
    import gsim
    scen = scen or {}
    k, T, D, Dlo, Dhi = cfg[1], cfg[2], cfg[3], cfg[4], cfg[5]
    net, beh = build_network((n,) + tuple(cfg[1:]), 2, scen)
    params = beacon_params(T)
    gp = gsim.GossipSubParams(D=D, Dlo=Dlo, Dhi=Dhi, PeerExchange=bool(scen.get("px")))
    if "opp_ticks" in scen:
        gp.OpportunisticGraftTicks = scen["opp_ticks"]
    rate = scen.get("msg_rate", MSG_RATE)
    lib = ob.load()
    all_threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))

    def leg(threads: int):
        got = lib.orc_set_threads(threads)
        st = ob.NetState(net, params, thresholds=beacon_thresholds(), gossip=gp)
        synthetic_state(st, np.random.default_rng(3), tick_time(0), D / k)   # gsim_fill_synthetic's distributions
        if "zipf_per_peer" in scen:
            restrict_to_subscriptions(st, net)
        ts = scen.get("topic_slots", 0)
        msgs = ob.Msgs(n, T, T * ts if ts else scen.get("ring", MSG_RING), ROUNDS, tick_time(0), SECOND,
                       behaviour=beh, topic_slots=ts)
        sched = message_schedule(n, T, range(1, ticks + 2), sub=net.sub if "zipf_per_peer" in scen else None,
                                 rate=rate)
        churn = churn_schedule(net, scen["churn_frac"], range(1, ticks + 2)) if "churn_frac" in scen else {}
        v = st.view()
        lib.orc_ip_colocation(v)
        times, deliv = [], []
        t_leg = time.perf_counter()
        for kk in range(1, ticks + 1 + warmup):
            now = tick_time(kk)
            d0 = msgs.stats[0]
            t0 = time.perf_counter()
            for (pairs, up) in churn.get(kk, []):
                st.churn(pairs, up=up, now=now - SECOND // 2)
            lib.orc_refresh_scores(v, now)
            msgs.penalties(st, now)
            lib.orc_compute_scores(v)
            msgs.heartbeat(st, kk, now, 0x5EED0001)
            for g in range(kk * ROUNDS, (kk + 1) * ROUNDS):
                for m in sched.get(g, []):
                    msgs.publish(st, int(m["id"]), int(m["topic"]), int(m["origin"]), 0, g)
                msgs.round(st, g)
            if gp.PeerExchange:
                st.px_connect(now + SECOND // 2)
            if kk > warmup:                             # the first `warmup` ticks warm up
                times.append(time.perf_counter() - t0)
                deliv.append(msgs.stats[0] - d0)
            if time.perf_counter() - t_leg > budget_s and len(times) >= 1:
                break
        med = float(np.median(times))
        return {"value": n / med, "cores": got, "ticks_timed": len(times), "median_tick_s": med,
                "msg_edge_deliveries_per_sec": float(np.median(deliv)) / med}

    one = leg(1) if "single" in legs else None
    allc = leg(all_threads) if "all" in legs else one
    lib.orc_set_threads(all_threads)
    n1 = one["ticks_timed"] if one else 0
    return {"value": allc["value"], "unit": "peer-heartbeat updates/sec", "cores": allc["cores"], "kind": "port",
            "msg_edge_deliveries_per_sec": allc["msg_edge_deliveries_per_sec"],
            "single_core": one, "all_core": allc,
            "sample": f"C oracle heartbeat tick (refreshScores+score, mesh maintenance, {ROUNDS} propagation "
                      f"rounds at {rate:g} msg/s/topic) on a {n}-peer {describe_graph(cfg, scen)}, T={T} "
                      f"network; median of {n1} (1 core) / {allc['ticks_timed']} "
                      f"({allc['cores']} OpenMP threads: refresh, score, heartbeat, control and the "
                      f"receivers of each propagation round) ticks after {warmup} warm-up tick(s)"}


def job_totals(wall: float, deliveries: float, dist=None, device: str = "cpu"):
    """Whole-job totals over the replica ranks: the slowest
    rank's wall time (MAX) and the deliveries of all ranks (SUM)."""
    if dist is None:
        return wall, deliveries
    import torch
    t = torch.tensor([wall, deliveries], device=device, dtype=torch.float64)
    w = t[:1].clone()
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
    d = t[1:].clone()
    dist.all_reduce(d, op=dist.ReduceOp.SUM)
    return float(w.item()), float(d.item())


def replica_seeds(rank: int):
    """Every rank simulates its own network: graph/state seed and message
    schedule seed differ per rank (weak scaling, no data-path collective)."""
    return 1 + rank, 2 + rank


def load_traffic(workload: str):
    path = os.path.join(REPO, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path)).get(workload)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-full", action="store_true",
                    help="time only the C oracle on the config's full network (no GPU): one tick per leg after "
                         "GSIM_CPU_WARMUP (1) warm-up ticks; GSIM_CPU_LEGS=all,single "
                         "(DESIGN.md §7); prints one JSON line")
    ap.add_argument("--msg-rate", type=float, default=None, help="messages per second per topic (config default)")
    ap.add_argument("--ring", type=int, default=None, help="message ring slots (config default)")
    ap.add_argument("--vdelay", type=int, default=0,
                    help="validation latency of every message in rounds (gsim_msg.vdelay)")
    ap.add_argument("--replicas", action="store_true",
                    help="N > 1: one independent network per rank (weak scaling) instead of one sharded network")
    ap.add_argument("--calltime", action="store_true",
                    help="diagnostic: print the wall ms per tick of each engine call (synchronised) to stderr")
    ap.add_argument("--peers", type=int, default=None,
                    help="peers of the config's network (its default otherwise): a reduced shape, e.g. c5 split "
                         "into 8 shards on one GPU, whose ghost rows would not fit its HBM at 10M peers")
    ap.add_argument("--shards", type=int, default=1,
                    help="N = 1: split the network into this many shards on the one GPU (exercises the halo "
                         "exchange through the in-process transport; not the headline configuration)")
    args = ap.parse_args()
    if args.cpu_full:
        cfg = CONFIGS[args.config]
        scen = dict(SCENARIOS.get(args.config, {}))
        legs = tuple(os.environ.get("GSIM_CPU_LEGS", "all,single").split(","))
        out = cpu_baseline(cfg, scen, n=cfg[0], ticks=1, budget_s=0.0,
                           warmup=int(os.environ.get("GSIM_CPU_WARMUP", "1")), legs=legs)
        out["config"] = args.config
        print(json.dumps(out), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    cfg = CONFIGS[args.config]
    if args.peers:
        cfg = (args.peers,) + tuple(cfg[1:])
    scen = dict(SCENARIOS.get(args.config, {}))
    if args.msg_rate is not None:
        scen["msg_rate"] = args.msg_rate
    if args.ring is not None:
        scen["ring"] = args.ring
    if args.vdelay:
        # slower propagation leaves more peers wanting at IHAVE time
        scen["max_arrivals"] = 64 * cfg[0]
    n, k, T = cfg[0], cfg[1], cfg[2]
    sharded = (world > 1 and not args.replicas) or args.shards > 1
    shard = None
    if args.shards > 1 and world == 1:
        g_seed, s_seed = replica_seeds(0)
        shard = args.shards
    elif sharded:
        # one network over every rank: same graph / schedule seeds, RCCL id from rank 0
        g_seed, s_seed = replica_seeds(0)
        from gsim.shard import ShardedEngine
        box = [ShardedEngine.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        shard = (rank, world, box[0])
    else:
        g_seed, s_seed = replica_seeds(rank)
    eng, net = build_engine(cfg, seed=g_seed, device=local, scen=scen, shard=shard)
    E = net.e
    hbm_used = None
    try:                                         # device memory in use once the state is resident
        import torch
        free_b, total_b = torch.cuda.mem_get_info(local)
        hbm_used = (total_b - free_b) / 1e9
    except Exception:
        pass
    ticks = range(1, args.warmup + args.steps + 1)
    rate = scen.get("msg_rate", MSG_RATE)
    sched = message_schedule(n, T, ticks, seed=s_seed, sub=net.sub if "zipf_per_peer" in scen else None, rate=rate)
    churn = churn_schedule(net, scen["churn_frac"], ticks, seed=s_seed + 2) if "churn_frac" in scen else None
    if args.vdelay:
        for arr in sched.values():
            arr["vdelay"] = args.vdelay

    kk = 0
    run_ticks(eng, kk, args.warmup, sched, churn, px=bool(scen.get("px")))
    kk += args.warmup
    eng.synchronize()
    census0 = eng.census()
    stats0 = eng.msg_stats()
    gossip0 = eng.gossip_stats()
    local_stats0 = eng.local_msg_stats() if sharded else stats0

    def barrier():
        if dist is not None:
            import torch
            t = torch.ones(1, device=f"cuda:{local}")
            dist.all_reduce(t)
            torch.cuda.synchronize()

    barrier()
    eng.profile(True)
    eng.synchronize()
    global CALLTIME
    if args.calltime:
        CALLTIME = {"_eng": eng}
    diag = _diag_phases(eng) if os.environ.get("GSIM_DIAG_PHASE") else None   # diagnostic builds only
    hb_diag = _diag_hb(eng) if os.environ.get("GSIM_DIAG_HB") else None
    ih_diag = _diag_ih(eng) if os.environ.get("GSIM_DIAG_IH") else None
    syncs0 = host_syncs(eng)
    t0 = time.perf_counter()
    run_ticks(eng, kk, args.steps, sched, churn, px=bool(scen.get("px")))
    kk += args.steps
    syncs1 = host_syncs(eng)
    eng.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    if diag:
        print(json.dumps({"send_phase_clocks_per_tick": [v / args.steps for v in diag()]}), file=sys.stderr)
    if hb_diag:
        print(json.dumps({"heartbeat_counts_per_tick": dict(zip(["rescored", "grafts", "prunes", "backoff_loads"],
                                                                 [v / args.steps for v in hb_diag()]))}),
              file=sys.stderr)
    if ih_diag:
        print(json.dumps({"ihave_counts_per_tick": {lp: {k: v / args.steps for k, v in d.items()}
                                                    for lp, d in ih_diag().items()}}), file=sys.stderr)
    if CALLTIME is not None:
        print(json.dumps({"calltime_ms_per_tick": {c: v / args.steps for c, v in CALLTIME.items() if c != "_eng"}}),
              file=sys.stderr)
        CALLTIME = None
    per_shard = None
    if shard is not None and world == 1:          # in-process shards: each one's kernel time
        per_shard = eng.profile_read_shards()
        prof = {c: (sum(p[c][0] for p in per_shard), sum(p[c][1] for p in per_shard)) for c in per_shard[0]}
    else:
        prof = eng.profile_read()
    eng.profile(False)
    local_stats1 = eng.local_msg_stats() if sharded else None
    census1 = eng.census()
    stats1 = eng.msg_stats()
    gossip1 = eng.gossip_stats()
    if sharded:
        # group totals are already the whole job's: only the wall time is reduced
        wall, _ = job_totals(wall, 0.0, dist, f"cuda:{local}")
        deliveries = float(stats1[0] - stats0[0])
    else:
        wall, deliveries = job_totals(wall, float(stats1[0] - stats0[0]), dist, f"cuda:{local}")

    if rank == 0:
        K = args.steps
        workload = (f"{args.config}: {n} peers{' (reduced: --peers)' if args.peers else ''}, "
                    f"{describe_graph(cfg, scen)}, {T} topics, beacon-style params, "
                    f"{rate:g} msg/s/topic, {ROUNDS} rounds/heartbeat")
        # peer-heartbeats of the whole job: one network (sharded) or one per rank
        value = n * (1 if sharded else world) * K / wall
        kms = {c: ms / K for c, (ms, _) in prof.items()}        # per tick
        launches = {c: cnt for c, (_, cnt) in prof.items()}
        # refresh+score: census-based compulsory bytes per launch
        alg_refresh = (refresh_bytes(census0, E) + refresh_bytes(census1, E)) // 2
        if sharded and world > 1:   # the kernels timed are rank 0's shard: its share of the network
            alg_refresh = alg_refresh // world
        elif per_shard is not None:  # in-process shards: ref_ms below is the average launch of ONE shard
            alg_refresh = alg_refresh // args.shards
        ref_ms = prof["refresh_score"][0] / max(1, launches["refresh_score"])
        ref_gbs = alg_refresh / (ref_ms * 1e-3) / 1e9
        # delivery: SURVEY.md §8(d) bytes per first / duplicate delivery, over send+commit(+accept)
        firsts = stats1[1] - stats0[1]
        dups = stats1[2] - stats0[2]
        if sharded:   # ... and the deliveries to its peers
            firsts, dups = (s1 - s0 for s1, s0 in zip(local_stats1[1:3], local_stats0[1:3]))
        alg_deliv = (FIRST_BYTES * firsts + DUP_BYTES * dups) / K
        deliv_ms = kms["send"] + kms["commit"] + kms["accept"]
        deliv_gbs = alg_deliv / (deliv_ms * 1e-3) / 1e9 if deliv_ms > 0 else 0.0
        # traffic: PMC HBM bytes (profiles/traffic.json), per launch like `achieved`
        # (measured on the default kernels: a --vdelay run uses other instances, so none is attached)
        tr_ref = None if args.vdelay else load_traffic(args.config)
        roof_refresh = {"bound": "hbm", "achieved": ref_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ref_gbs / HBM_PEAK_GBS,
                        "traffic": tr_ref["bytes_per_launch"] if tr_ref else None, "traffic_detail": tr_ref,
                        "kernel": "k_refresh_score<true,true>", "kernel_ms": ref_ms,
                        "algorithmic_bytes_per_launch": alg_refresh}
        # PMC traffic of k_send (per launch) scaled to a tick, the unit delivery's bytes are quoted in
        tr_send = None if args.vdelay else load_traffic(args.config + ":send")
        tr_send_tick = None
        if tr_send is not None:
            tr_send_tick = tr_send["bytes_per_launch"] * launches["send"] / K
            tr_send = dict(tr_send, bytes_per_tick=tr_send_tick, covers="k_send_tm + k_commit")
        roof_deliv = {"bound": "hbm", "achieved": deliv_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": deliv_gbs / HBM_PEAK_GBS, "traffic": tr_send_tick, "traffic_detail": tr_send,
                      "kernel": "delivery: k_send_tm + k_commit + k_delivery_state (per tick, 10 rounds)", "kernel_ms": deliv_ms,
                      "algorithmic_bytes_per_tick": alg_deliv}
        # the delivery walk against the random-access probes (profiles/r01_probe_random_access.jsonl):
        # its L2 misses against random 8-B loads over a 2 GB table (every one a miss, 54 G/s), and
        # all its TCC requests against the same loads over an L2-resident 4 MB table (251 G/s) --
        # two ceilings a request stream cannot pass, so neither fraction can exceed 1
        rq = None if args.vdelay or sharded else load_traffic(args.config + ":send_req")
        if rq is not None and launches.get("send"):
            send_launch_ms = kms["send"] * K / launches["send"]
            copies_per_launch = (firsts + dups) / launches["send"] if launches["send"] else 0
            req_s = rq["requests_per_launch"] / (send_launch_ms * 1e-3)
            miss_s = rq["tcc_miss"] / (send_launch_ms * 1e-3)
            roof_deliv["request_bounds"] = {
                "kernel": rq["kernel"], "kernel_ms_per_launch": send_launch_ms, "source": rq["source"],
                "copies_per_launch": copies_per_launch,
                "l2_misses": {"bound": "random_miss_rate", "achieved": miss_s, "peak": PROBE_MISS_PER_S,
                              "unit": "requests/s", "frac": miss_s / PROBE_MISS_PER_S,
                              "per_launch": rq["tcc_miss"], "per_copy": rq["tcc_miss"] / max(1, copies_per_launch),
                              "peak_source": "random 8-B loads, 2 GB table (L2 misses): 54.1 G/s"},
                "tcc_requests": {"bound": "l2_request_rate", "achieved": req_s, "peak": PROBE_L2_REQ_PER_S,
                                 "unit": "requests/s", "frac": req_s / PROBE_L2_REQ_PER_S,
                                 "per_launch": rq["requests_per_launch"],
                                 "per_copy": rq["requests_per_launch"] / max(1, copies_per_launch),
                                 "l2_hit_rate": rq.get("hit_rate"),
                                 "peak_source": "random 8-B loads, L2-resident 4 MB table: 251 G/s"},
                "probe": "profiles/r01_probe_random_access.jsonl"}
        # the heartbeat's bound: VALU issue (PMC SQ_INSTS_VALU per launch of k_heartbeat<32>) over
        # the heartbeat class's time per tick (it also holds k_fanout_heartbeat: a slight under-estimate)
        hv = None if args.vdelay or sharded else load_traffic(args.config + ":hb_valu")
        roof_hb = None
        if hv is not None and kms.get("heartbeat"):
            ach = hv["valu_insts_per_launch"] / (kms["heartbeat"] * 1e-3)
            roof_hb = {"bound": "valu_issue", "achieved": ach, "peak": hv["peak_wave_insts_per_s"],
                       "unit": "wave-instructions/s", "frac": ach / hv["peak_wave_insts_per_s"],
                       "valu_insts_per_launch": hv["valu_insts_per_launch"],
                       "valu_insts_per_peer_topic": hv["valu_insts_per_launch"] / (n * T),
                       "kernel": hv["kernel"] + " (+ k_fanout_heartbeat in kernel_ms)", "kernel_ms": kms["heartbeat"],
                       "source": hv["source"], "peak_source": hv["peak_source"]}
            if hv.get("salu_insts_per_launch"):
                # the scalar unit: one SALU instruction per cycle per CU (shared by its 4 SIMDs)
                s_ach = hv["salu_insts_per_launch"] / (kms["heartbeat"] * 1e-3)
                s_peak = SALU_PEAK
                roof_hb["salu_issue"] = {"bound": "salu_issue", "achieved": s_ach, "peak": s_peak,
                                         "unit": "instructions/s", "frac": s_ach / s_peak,
                                         "salu_insts_per_launch": hv["salu_insts_per_launch"],
                                         "peak_source": "256 CUs x 2.4 GHz, one scalar issue per CU per cycle"}
        dominant = roof_refresh if ref_ms * launches["refresh_score"] / K >= deliv_ms else roof_deliv
        out = {
            "metric": "peer-heartbeat updates/sec + msg-edge deliveries/sec, 1M-peer gossipsub sim",
            "value": value,
            "unit": "peer-heartbeat updates/sec",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": wall / K * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (seeded {'power-law' if 'power_law' in scen else 'random-regular'} graph, "
                    "Philox-seeded steady-state counters and meshes, Poisson message publications)",
            "config": {"workload": workload, "peers_per_gpu": n, "degree": k, "topics": T,
                       "edge_topic_records": E * T, "rounds_per_heartbeat": ROUNDS,
                       "max_degree": int(np.diff(net.row_ptr.astype(np.int64)).max()),
                       "hbm_used_gb": hbm_used,
                       "step": "heartbeat tick: refreshScores+score, mesh maintenance, "
                               f"{ROUNDS} propagation rounds (publish, deliver, control, forward)",
                       "parallelism": (f"graph-sharded x{world} (RCCL halo exchange)" if sharded and world > 1
                                       else f"graph-sharded x{args.shards} on one GPU (in-process exchange)"
                                       if sharded else f"replica-per-gpu x{world}"),
                       **({"validation_latency_rounds": args.vdelay} if args.vdelay else {})},
            "msg_edge_deliveries_per_sec": deliveries / wall,
            "deliveries_per_tick": {"accepted": (stats1[0] - stats0[0]) / K, "first": (stats1[1] - stats0[1]) / K,
                                    "duplicate": (stats1[2] - stats0[2]) / K, "graylisted": (stats1[3] - stats0[3]) / K},
            "kernel_ms_per_tick": kms,
            # in-process shards (GSIM_GROUP_SERIAL=1: each alone on the device): kernel ms per tick of each
            "kernel_ms_per_tick_shards": (None if per_shard is None else
                                          [round(sum(ms for ms, _ in p.values()) / K, 3) for p in per_shard]),
            # strong scaling is set by the slowest shard (each alone on the device, in-process
            # exchange): per-tick kernel ms of the max and mean shard
            "shard_kernel_ms_per_tick": (None if per_shard is None else {
                "max": max(sum(ms for ms, _ in p.values()) for p in per_shard) / K,
                "mean": sum(sum(ms for ms, _ in p.values()) for p in per_shard) / len(per_shard) / K,
                "summed": sum(sum(ms for ms, _ in p.values()) for p in per_shard) / K}),
            "gossip_per_tick": {k: (gossip1[k] - gossip0[k]) / K for k in gossip1},
            "box": box_info(),
            # host round trips inside the timed ticks (stream synchronisations and blocking
            # copies the library made, per tick)
            "host_syncs_per_tick": (syncs1 - syncs0) / K,
            "census": census1,
            "roofline": dominant,
            "roofline_kernels": {"refresh_score": roof_refresh, "delivery": roof_deliv,
                                 **({"heartbeat": roof_hb} if roof_hb else {})},
        }
        if not args.no_cpu_baseline and world == 1 and not args.vdelay:
            # (the oracle baseline publishes without latency: not the same workload as a --vdelay line)
            out["cpu_baseline"] = cpu_baseline(cfg, scen=scen)
            # the same oracle on the whole network, timed on a GPU box's host cores by
            # `bench.py --cpu-full` (minutes per tick: not re-run here)
            full = os.path.join(REPO, "profiles", f"cpu_full_{args.config}_box16.json")
            if os.path.exists(full):
                try:
                    fd = json.loads(open(full).read().strip().splitlines()[-1])
                    out["cpu_baseline"]["full_network"] = {
                        "value": fd["value"], "cores": fd["cores"], "median_tick_s": fd["all_core"]["median_tick_s"],
                        "msg_edge_deliveries_per_sec": fd["msg_edge_deliveries_per_sec"],
                        "gpu_over_cpu": value / fd["value"], "source": os.path.relpath(full, REPO)}
                except (OSError, ValueError, KeyError):
                    pass
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
