#!/usr/bin/env python3
"""Turn rocprofv3 --pmc counter CSVs into per-launch HBM traffic for bench.py.

Two separate passes (MI355X_MICROARCH.md §rocprofv3 PMC slots: FETCH_SIZE and
WRITE_SIZE cannot share a pass):
  rocprofv3 --pmc FETCH_SIZE ... -> <dir_fetch>/*counter_collection.csv
  rocprofv3 --pmc WRITE_SIZE ... -> <dir_write>/*counter_collection.csv
Both counters are in KiB.  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE reads exactly half the bytes of a wide coalesced streaming read, so
the read side is doubled; WRITE_SIZE is exact for streaming stores.  The
corrected value and the raw counters are both recorded.

usage: pmc_traffic.py <workload-id> <kernel-regex> <fetch_dir> <write_dir> [out.json]
"""
import csv
import glob
import json
import os
import re
import sys


def per_launch(directory, counter, kernel_re):
    vals = []
    for path in glob.glob(os.path.join(directory, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name") or row.get("KernelName") or ""
                if not re.search(kernel_re, name):
                    continue
                if row.get("Counter_Name", counter) != counter:
                    continue
                vals.append(float(row.get("Counter_Value") or row.get(counter)))
    return vals


def main():
    workload, kre, dfetch, dwrite = sys.argv[1:5]
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "traffic.json")
    f = per_launch(dfetch, "FETCH_SIZE", kre)
    w = per_launch(dwrite, "WRITE_SIZE", kre)
    if not f or not w:
        raise SystemExit(f"no samples (fetch {len(f)}, write {len(w)})")
    fk = sum(f) / len(f)
    wk = sum(w) / len(w)
    rec = {"bytes_per_launch": (2 * fk + wk) * 1024, "fetch_kib_raw": fk, "write_kib_raw": wk,
           "launches": [len(f), len(w)], "kernel_regex": kre,
           "correction": "read side x2 (gfx950 FETCH_SIZE under-count), write exact"}
    if workload.endswith(":send"):
        rec["calibration"] = ("k_send's accesses are 1-8 B gathers and atomics at random addresses; the x2 "
                              "read correction is calibrated for 16-B/lane streaming reads only")
    data = {}
    if os.path.exists(out):
        data = json.load(open(out))
    data[workload] = rec
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps({workload: rec}))


if __name__ == "__main__":
    main()
