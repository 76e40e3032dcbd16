#!/usr/bin/env python3
"""A/B timing of kernel variants (gsim_set_kernel_variant(h, which, v)) on the
C3 workload.  Results are identical across variants; each arm runs whole ticks
and the per-tick kernel times are compared.  Arms are interleaved.
usage: python tools/ab_variants.py --which 4 --variants 1,2 [--rounds 3] [--ticks 2]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", type=int, default=2)
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ticks", type=int, default=2)
    args = ap.parse_args()
    arms = [int(x) for x in args.variants.split(",")]
    cfg = bench.CONFIGS["c3"]
    eng, net = bench.build_engine(cfg, seed=1, device=0)
    total = 3 + args.rounds * len(arms) * args.ticks
    sched = bench.message_schedule(cfg[0], cfg[2], range(1, total + 2))
    k = 0
    for _ in range(3):
        k += 1
        bench.run_tick(eng, k, sched)
    times = {a: [] for a in arms}
    for _ in range(args.rounds):
        for v in arms:
            eng.set_kernel_variant(args.which, v)
            eng.profile(True)
            for _ in range(args.ticks):
                k += 1
                bench.run_tick(eng, k, sched)
            prof = eng.profile_read()
            eng.profile(False)
            times[v].append({c: ms / args.ticks for c, (ms, _) in prof.items() if ms > 0})
    out = {}
    for v, runs in times.items():
        out[f"variant_{v}"] = {c: round(float(np.median([x.get(c, 0.0) for x in runs])), 3) for c in runs[0]}
    print(json.dumps({"which": args.which, "kernel_ms_per_tick_median": out}))
    eng.close()


if __name__ == "__main__":
    main()
