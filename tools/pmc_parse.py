#!/usr/bin/env python3
"""Per-kernel, per-launch PMC counter means from rocprofv3 --pmc passes.

usage: pmc_parse.py OUT.json DIR [DIR ...]

Every DIR holds one pass (`rocprofv3 --pmc ... -d DIR`).  Counter rows of one
dispatch are summed (one row per XCD / SE instance), then averaged over the
kernel's steady launches: the first third of each kernel's launches (the
bench's warm-up tick) is dropped.  The kernel key is the template name before
the argument list (e.g. "k_send_tm<1024, false, false, false, false>").
"""
import collections
import csv
import glob
import json
import os
import sys


def kernel_key(name: str) -> str:
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    depth, out = 0, []
    for ch in name:                       # cut at the '(' of the argument list, outside <...>
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out)


def parse(dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                k = kernel_key(r.get("Kernel_Name", ""))
                per[k][int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for k, disp in per.items():
        ids = sorted(disp)
        counters = collections.defaultdict(list)
        for i in ids:
            for c, v in disp[i].items():
                counters[c].append(v)
        rec = {}
        for c, vals in counters.items():
            steady = vals[len(vals) // 3:] or vals
            rec[c] = sum(steady) / len(steady)
        rec["_launches"] = len(ids)
        out[k] = rec
    return out


def main():
    out = parse(sys.argv[2:])
    json.dump(out, open(sys.argv[1], "w"), indent=1, sort_keys=True)
    for k, rec in sorted(out.items()):
        print(k)
        for c, v in sorted(rec.items()):
            print(f"   {c:36s} {v:.5g}")


if __name__ == "__main__":
    main()
