#!/usr/bin/env python3
"""Ablation timing of the delivery kernel (k_send) on the C3 workload.

Each arm runs whole ticks (refresh, heartbeat, 10 rounds) with one cost of
k_send removed (gsim_set_kernel_variant(h, 1, mask)); results are wrong by
construction and only the per-tick k_send time is meaningful.  Arms are
interleaved over several rounds in one process.
usage: python tools/ab_deliver.py [--rounds 3] [--ticks 2]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

ARMS = {0: "full", 32768: "hb_wave_rows", 512: "hb_no_gossip"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ticks", type=int, default=2)
    args = ap.parse_args()
    cfg = bench.CONFIGS["c3"]
    eng, net = bench.build_engine(cfg, seed=1, device=0)
    total = 3 + args.rounds * len(ARMS) * args.ticks
    sched = bench.message_schedule(cfg[0], cfg[2], range(1, total + 2))
    k = 0
    for _ in range(3):
        k += 1
        bench.run_tick(eng, k, sched)
    times = {a: [] for a in ARMS}
    for _ in range(args.rounds):
        for d in ARMS:
            eng.set_kernel_variant(1, d)
            eng.profile(True)
            for _ in range(args.ticks):
                k += 1
                bench.run_tick(eng, k, sched)
            prof = eng.profile_read()
            eng.profile(False)
            times[d].append({c: ms / args.ticks for c, (ms, _) in prof.items() if ms > 0})
    eng.set_kernel_variant(1, 0)
    out = {}
    for d, v in times.items():
        out[ARMS[d]] = {c: round(float(np.median([x.get(c, 0.0) for x in v])), 3) for c in v[0]}
    print(json.dumps({"kernel_ms_per_tick_median": out, "gossip_per_run": eng.gossip_stats()}))
    eng.close()


if __name__ == "__main__":
    main()
