#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line: tools/bench_summary.py FILE"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(round(d["ms_per_step"], 2), "ms/tick", f"{d['value']:.4g}", d["unit"], "frac", round(d["roofline"]["frac"], 4))
print(d["config"]["workload"])
print({k: round(v, 2) for k, v in d["kernel_ms_per_tick"].items() if v > 0.05})
cb = d.get("cpu_baseline")
if cb:
    print("cpu", f"{cb['value']:.4g}", "all-core;", f"{cb['single_core']['value']:.4g}", "single-core")
