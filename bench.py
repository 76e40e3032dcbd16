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

Multi-GPU: each rank simulates its own 1M-peer network on its own GPU (weak
scaling, "replicas only" until the sharded halo-exchange path lands;
DESIGN.md §5).
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
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
ROUNDS = 10                    # propagation rounds per heartbeat
MSG_RATE = 4.0                 # messages / s / topic
MSG_RING = 1024                # live-message window: >= 16 heartbeats of publications, so no slot
                               # is republished while its message can still be gossiped or promised
DUP_BYTES, FIRST_BYTES = 40, 72   # algorithmic bytes per delivery

CONFIGS = {
    # id: (peers, degree, topics, D, Dlo, Dhi)
    "c3": (1_000_000, 32, 16, 8, 6, 12),
    "c2": (10_000, 32, 1, 8, 6, 12),
}


def refresh_bytes(census: dict, n_edges: int) -> int:
    """Compulsory HBM bytes of one refreshScores+score pass on this state
    (DESIGN.md §4.1): every connected scored record reads its 4 counters and
    flags (33 B); in-mesh records also read graftTime and write meshTime
    (16 B); every non-zero counter changes under decay and is written (8 B);
    per edge: estate 1, bp r+w 16, P5 gather 8, col 4, P6 8, score write 8."""
    nz = census["nz_first"] + census["nz_meshd"] + census["nz_fail"] + census["nz_invalid"]
    return 33 * census["records"] + 16 * census["in_mesh"] + 8 * nz + 45 * n_edges


def tick_time(k: int) -> int:
    return 3600 * SECOND + k * SECOND


def message_schedule(n: int, T: int, ticks: range, seed: int = 2) -> dict:
    """{round: gsim_msg array}: Poisson(MSG_RATE) messages per topic per
    heartbeat, each in a uniform round of its tick, origin uniform."""
    from gsim import _abi
    rng = np.random.default_rng(seed)
    out, mid = {}, 0
    for k in ticks:
        per_round = [[] for _ in range(ROUNDS)]
        for t in range(T):
            for _ in range(rng.poisson(MSG_RATE)):
                per_round[int(rng.integers(0, ROUNDS))].append((mid, t, int(rng.integers(0, n))))
                mid += 1
        for r, lst in enumerate(per_round):
            if lst:
                a = np.zeros(len(lst), dtype=_abi.MSG_DTYPE)
                a["id"] = [x[0] for x in lst]
                a["topic"] = [x[1] for x in lst]
                a["origin"] = [x[2] for x in lst]
                out[k * ROUNDS + r] = a
    return out


def build_engine(cfg, seed, device):
    import gsim
    from gsim.presets import beacon_params, beacon_thresholds
    n, k, T, D, Dlo, Dhi = cfg
    params = beacon_params(T)
    gp = gsim.GossipSubParams(D=D, Dlo=Dlo, Dhi=Dhi)
    eng = gsim.Engine(params, beacon_thresholds(), gossip=gp, device=device)
    net = gsim.random_regular(n, k, seed=seed, n_topics=T)
    eng.load_graph(net)
    eng.set_seed(0x5EED0000 + seed)
    eng.fill_synthetic(seed=seed * 7919 + 1, now=tick_time(0), p_mesh=D / k)
    eng.msgs_init(MSG_RING, ROUNDS, tick_time(0), SECOND)
    if os.environ.get("GSIM_SEND_VARIANT"):          # A/B of the delivery kernel variants (gsim.h)
        eng.set_kernel_variant(2, int(os.environ["GSIM_SEND_VARIANT"]))
    return eng, net


def run_tick(eng, k, sched):
    now = tick_time(k)
    eng.refresh_scores(now)
    eng.heartbeat(k, now)
    for g in range(k * ROUNDS, (k + 1) * ROUNDS):
        m = sched.get(g)
        if m is not None:
            eng.publish_array(m, g)
        eng.round(g)


def cpu_baseline(cfg, budget_s: float = 15.0):
    """Time the C oracle (OpenMP over observers in the heartbeat phases) on a
    bounded sample of the same workload: same degree, topics, parameters and
    message rate, 50k peers."""
    import oracle_binding as ob
    from fixtures import beacon_params, beacon_thresholds, synthetic_state
    import gsim
    n, k, T, D, Dlo, Dhi = 50_000, cfg[1], cfg[2], cfg[3], cfg[4], cfg[5]
    net = gsim.random_regular(n, k, seed=2, n_topics=T)
    params = beacon_params(T)
    st = ob.NetState(net, params, thresholds=beacon_thresholds(), gossip=gsim.GossipSubParams(D=D, Dlo=Dlo, Dhi=Dhi))
    synthetic_state(st, np.random.default_rng(3), tick_time(0), D / k)   # gsim_fill_synthetic's distributions
    msgs = ob.Msgs(n, T, MSG_RING, ROUNDS, tick_time(0), SECOND)
    sched = message_schedule(n, T, range(1, 201))
    lib = ob.load()
    v = st.view()
    lib.orc_ip_colocation(v)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    steps = 0
    t0 = time.perf_counter()
    while True:
        kk = steps + 1
        now = tick_time(kk)
        lib.orc_refresh_scores(v, now)
        msgs.penalties(st, now)
        lib.orc_compute_scores(v)
        msgs.heartbeat(st, kk, now, 0x5EED0001)
        for g in range(kk * ROUNDS, (kk + 1) * ROUNDS):
            for m in sched.get(g, []):
                msgs.publish(st, int(m["id"]), int(m["topic"]), int(m["origin"]), 0, g)
            msgs.round(st, g)
        steps += 1
        if time.perf_counter() - t0 > budget_s or steps >= 200:
            break
    el = time.perf_counter() - t0
    return {"value": n * steps / el, "unit": "peer-heartbeat updates/sec", "cores": threads, "kind": "port",
            "msg_edge_deliveries_per_sec": msgs.stats[0] / el,
            "sample": f"C oracle heartbeat tick (refreshScores+score, mesh maintenance, {ROUNDS} propagation "
                      f"rounds at {MSG_RATE:g} msg/s/topic) on a {n}-peer k={k} T={T} network, {steps} ticks, "
                      f"OpenMP {threads} threads in the heartbeat phases, {el:.1f}s"}


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
    args = ap.parse_args()

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
    n, k, T = cfg[0], cfg[1], cfg[2]
    g_seed, s_seed = replica_seeds(rank)
    eng, net = build_engine(cfg, seed=g_seed, device=local)
    E = net.e
    sched = message_schedule(n, T, range(1, args.warmup + args.steps + 1), seed=s_seed)

    kk = 0
    for _ in range(args.warmup):
        kk += 1
        run_tick(eng, kk, sched)
    eng.synchronize()
    census0 = eng.census()
    stats0 = eng.msg_stats()
    gossip0 = eng.gossip_stats()

    def barrier():
        if dist is not None:
            import torch
            t = torch.ones(1, device=f"cuda:{local}")
            dist.all_reduce(t)
            torch.cuda.synchronize()

    barrier()
    eng.profile(True)
    eng.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        kk += 1
        run_tick(eng, kk, sched)
    eng.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    prof = eng.profile_read()
    eng.profile(False)
    census1 = eng.census()
    stats1 = eng.msg_stats()
    gossip1 = eng.gossip_stats()
    wall, deliveries = job_totals(wall, float(stats1[0] - stats0[0]), dist, f"cuda:{local}")

    if rank == 0:
        K = args.steps
        workload = (f"{args.config}: {n} peers, random-regular k={k}, {T} topics, beacon-style params, "
                    f"{MSG_RATE:g} msg/s/topic, {ROUNDS} rounds/heartbeat")
        value = n * world * K / wall
        kms = {c: ms / K for c, (ms, _) in prof.items()}        # per tick
        launches = {c: cnt for c, (_, cnt) in prof.items()}
        # refresh+score: census-based compulsory bytes per launch
        alg_refresh = (refresh_bytes(census0, E) + refresh_bytes(census1, E)) // 2
        ref_ms = prof["refresh_score"][0] / max(1, launches["refresh_score"])
        ref_gbs = alg_refresh / (ref_ms * 1e-3) / 1e9
        # delivery: SURVEY.md §8(d) bytes per first / duplicate delivery, over send+commit(+accept)
        firsts = stats1[1] - stats0[1]
        dups = stats1[2] - stats0[2]
        alg_deliv = (FIRST_BYTES * firsts + DUP_BYTES * dups) / K
        deliv_ms = kms["send"] + kms["commit"] + kms["accept"]
        deliv_gbs = alg_deliv / (deliv_ms * 1e-3) / 1e9 if deliv_ms > 0 else 0.0
        roof_refresh = {"bound": "hbm", "achieved": ref_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ref_gbs / HBM_PEAK_GBS, "traffic": load_traffic(args.config),
                        "kernel": "k_refresh_score<true,true>", "kernel_ms": ref_ms,
                        "algorithmic_bytes_per_launch": alg_refresh}
        # PMC traffic of k_send (profiles/traffic.json, per launch) scaled to a tick
        tr_send = load_traffic(args.config + ":send")
        if tr_send is not None:
            per_tick = tr_send["bytes_per_launch"] * launches["send"] / K
            tr_send = dict(tr_send, bytes_per_tick=per_tick)
        roof_deliv = {"bound": "hbm", "achieved": deliv_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": deliv_gbs / HBM_PEAK_GBS, "traffic": tr_send,
                      "kernel": "delivery: k_send_tm + k_commit + k_delivery_state (per tick, 10 rounds)", "kernel_ms": deliv_ms,
                      "algorithmic_bytes_per_tick": alg_deliv}
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded random-regular graph, Philox-seeded steady-state counters and meshes, "
                    "Poisson message publications)",
            "config": {"workload": workload, "peers_per_gpu": n, "degree": k, "topics": T,
                       "edge_topic_records": E * T, "rounds_per_heartbeat": ROUNDS,
                       "step": "heartbeat tick: refreshScores+score, mesh maintenance, "
                               f"{ROUNDS} propagation rounds (publish, deliver, control, forward)",
                       "parallelism": f"replica-per-gpu x{world}"},
            "msg_edge_deliveries_per_sec": deliveries / wall,
            "deliveries_per_tick": {"accepted": (stats1[0] - stats0[0]) / K, "first": firsts / K,
                                    "duplicate": dups / K, "graylisted": (stats1[3] - stats0[3]) / K},
            "kernel_ms_per_tick": kms,
            "gossip_per_tick": {k: (gossip1[k] - gossip0[k]) / K for k in gossip1},
            "census": census1,
            "roofline": dominant,
            "roofline_kernels": {"refresh_score": roof_refresh, "delivery": roof_deliv},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
