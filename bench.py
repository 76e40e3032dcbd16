#!/usr/bin/env python3
"""bench.py — peer-heartbeat updates/sec on the 1M-peer, 16-topic network (C3).

A "step" is one heartbeat tick of the whole simulated network with every byte
of state resident in HBM:
  refreshScores+score (decay, P1-P7 snapshot)  -> k_refresh_score_tile
  heartbeat mesh maintenance (all peers/topics) -> k_heartbeat
  control rounds 0 and 1 (GRAFT/PRUNE handling) -> k_handle_control x2
W untimed warmup ticks, then exactly K timed ticks bracketed by barrier +
device sync; max over ranks; rank 0 prints one JSON line.

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


def build_engine(cfg, seed, device):
    import gsim
    from fixtures import beacon_params, beacon_thresholds
    n, k, T, D, Dlo, Dhi = cfg
    params = beacon_params(T)
    gp = gsim.GossipSubParams(D=D, Dlo=Dlo, Dhi=Dhi)
    eng = gsim.Engine(params, beacon_thresholds(), gossip=gp, device=device)
    net = gsim.random_regular(n, k, seed=seed, n_topics=T)
    eng.load_graph(net)
    eng.set_seed(0x5EED0000 + seed)
    eng.fill_synthetic(seed=seed * 7919 + 1, now=tick_time(0), p_mesh=D / k)
    return eng, net


def run_tick(eng, k):
    now = tick_time(k)
    dt = SECOND // (ROUNDS + 1)
    eng.refresh_scores(now)
    eng.heartbeat(k, now)
    eng.handle_control(0, now + dt)
    eng.handle_control(1, now + 2 * dt)


def cpu_baseline(cfg, budget_s: float = 15.0):
    """Time the C oracle (OpenMP over observers) on a bounded sample of the
    same workload: same degree, topics and parameters, 50k peers."""
    import oracle_binding as ob
    from fixtures import beacon_params, beacon_thresholds, randomize_state
    import gsim
    n, k, T, D, Dlo, Dhi = 50_000, cfg[1], cfg[2], cfg[3], cfg[4], cfg[5]
    net = gsim.random_regular(n, k, seed=2, n_topics=T)
    params = beacon_params(T)
    st = ob.NetState(net, params, thresholds=beacon_thresholds(), gossip=gsim.GossipSubParams(D=D, Dlo=Dlo, Dhi=Dhi))
    rng = np.random.default_rng(3)
    randomize_state(st, rng, tick_time(0), retained_frac=0.0)
    st.tflags[...] = np.where(rng.random(st.tflags.shape) < D / k, 0x05, 0).astype(np.uint8)
    lib = ob.load()
    v = st.view()
    lib.orc_ip_colocation(v)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    steps = 0
    dt = SECOND // (ROUNDS + 1)
    t0 = time.perf_counter()
    while True:
        kk = steps + 1
        now = tick_time(kk)
        lib.orc_refresh_scores(v, now)
        lib.orc_compute_scores(v)
        lib.orc_heartbeat(v, kk, now, 0x5EED0001)
        lib.orc_handle_control(v, 0, now + dt)
        lib.orc_handle_control(v, 1, now + 2 * dt)
        steps += 1
        if time.perf_counter() - t0 > budget_s or steps >= 200:
            break
    el = time.perf_counter() - t0
    return {"value": n * steps / el, "unit": "peer-heartbeat updates/sec", "cores": threads, "kind": "port",
            "sample": f"C oracle heartbeat tick (refreshScores+score, mesh maintenance, 2 control rounds) on a "
                      f"{n}-peer k={k} T={T} network, {steps} ticks, OpenMP {threads} threads, {el:.1f}s"}


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
    if args.steps * 3 + 1 > 512:
        raise SystemExit("--steps must be <= 170 (event pool)")

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
    eng, net = build_engine(cfg, seed=1 + rank, device=local)
    E = net.e

    kk = 0
    for _ in range(args.warmup):
        kk += 1
        run_tick(eng, kk)
    eng.synchronize()
    census0 = eng.census()

    def barrier():
        if dist is not None:
            import torch
            t = torch.ones(1, device=f"cuda:{local}")
            dist.all_reduce(t)
            torch.cuda.synchronize()

    barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    dt = SECOND // (ROUNDS + 1)
    for s in range(args.steps):
        kk += 1
        now = tick_time(kk)
        eng.event_record(3 * s)
        eng.refresh_scores(now)
        eng.event_record(3 * s + 1)
        eng.heartbeat(kk, now)
        eng.event_record(3 * s + 2)
        eng.handle_control(0, now + dt)
        eng.handle_control(1, now + 2 * dt)
    eng.event_record(3 * args.steps)
    eng.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    ph = np.zeros(3)
    for s in range(args.steps):
        ph += [eng.event_elapsed_ms(3 * s + j, 3 * s + j + 1) for j in range(3)]
    ph /= args.steps
    census1 = eng.census()
    if dist is not None:
        import torch
        t = torch.tensor([wall], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    if rank == 0:
        workload = f"{args.config}: {n} peers, random-regular k={k}, {T} topics, beacon-style params"
        value = n * world * args.steps / wall
        alg = (refresh_bytes(census0, E) + refresh_bytes(census1, E)) // 2
        refresh_ms = float(ph[0])
        achieved = alg / (refresh_ms * 1e-3) / 1e9
        out = {
            "metric": "peer-heartbeat updates/sec + msg-edge deliveries/sec, 1M-peer gossipsub sim",
            "value": value,
            "unit": "peer-heartbeat updates/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded random-regular graph, Philox-seeded steady-state counters and meshes)",
            "config": {"workload": workload, "peers_per_gpu": n, "degree": k, "topics": T,
                       "edge_topic_records": E * T,
                       "step": "heartbeat tick: refreshScores+score, mesh maintenance, 2 control rounds",
                       "parallelism": f"replica-per-gpu x{world}"},
            "phases_ms": {"refresh_score": refresh_ms, "heartbeat": float(ph[1]), "control_rounds": float(ph[2])},
            "census": census1,
            "msg_edge_deliveries_per_sec": None,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(args.config),
                         "kernel": "k_refresh_score_tile<true,true>", "kernel_ms": refresh_ms,
                         "algorithmic_bytes_per_launch": alg},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
