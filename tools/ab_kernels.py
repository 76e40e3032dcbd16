#!/usr/bin/env python3
"""In-process A/B timing of hot-path kernel variants on the C3 workload
(cdna_hip_programming.md §5.4 rule 24: interleaved rounds in one process).

usage: python tools/ab_kernels.py [--rounds 5] [--iters 5] [--config c3] [--diag]
Prints one JSON line: per-variant median/min ms of the refresh+score pass
(and, with --diag, of ablations that drop one cost at a time — their results
are wrong by construction and only their time is meaningful), plus the
heartbeat / control-round phases of a full tick.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

VARIANTS = {0: "thread", 1: "pipe", 2: "wave4", 3: "wave8"}
DIAGS = {0: "full", 1: "no_p5_gather", 2: "no_mtime_store", 4: "no_stores", 8: "no_graft_load", 16: "no_p1_div",
         4 | 8 | 1: "loads_only(no graft,no p5)", 65536: "no_unjoined_skip"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--diag", action="store_true")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    eng, net = bench.build_engine(cfg, seed=1, device=0)
    sched = bench.message_schedule(cfg[0], cfg[2], range(1, 4))
    k = 0
    for _ in range(3):                       # settle the meshes
        k += 1
        bench.run_tick(eng, k, sched)
    census = eng.census()
    arms = [(v, 0) for v in VARIANTS] + [(0, 65536), (1, 65536)]
    if args.diag:
        arms += [(2, d) for d in DIAGS if d]
    times = {a: [] for a in arms}
    for _ in range(args.rounds):
        for (v, d) in arms:
            eng.set_kernel_variant(0, v)
            eng.set_kernel_variant(1, d)
            eng.synchronize()
            eng.event_record(0)
            for _ in range(args.iters):
                k += 1
                eng.refresh_scores(bench.tick_time(k))
            eng.event_record(1)
            times[(v, d)].append(eng.event_elapsed_ms(0, 1) / args.iters)
    eng.set_kernel_variant(0, 2)
    eng.set_kernel_variant(1, 0)
    ph = []
    for _ in range(args.iters):
        k += 1
        now = bench.tick_time(k)
        dt = bench.SECOND // (bench.ROUNDS + 1)
        eng.event_record(0)
        eng.refresh_scores(now)
        eng.event_record(1)
        eng.heartbeat(k, now)
        eng.event_record(2)
        eng.handle_control(0, now + dt)
        eng.handle_control(1, now + 2 * dt)
        eng.event_record(3)
        ph.append([eng.event_elapsed_ms(j, j + 1) for j in range(3)])
    alg = bench.refresh_bytes(census, net.e)
    out = {"refresh_ms": {f"{VARIANTS[v]}/{DIAGS[d]}": {"median": float(np.median(t)), "min": float(np.min(t))}
                          for (v, d), t in times.items()},
           "alg_bytes": alg,
           "alg_GBps_median_full": {VARIANTS[v]: alg / (float(np.median(times[(v, 0)])) * 1e-3) / 1e9
                                    for v in VARIANTS},
           "tick_phases_ms_median": [float(x) for x in np.median(np.array(ph), axis=0)],
           "census": census}
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
