"""Summarise a rocprofv3 kernel trace (csv): per-kernel time per tick per
shard over the timed ticks (the warmup tick's dispatches are dropped: the
trace starts at the (shards+1)-th refresh dispatch, one per tick and shard)."""
import collections
import csv
import sys


def main(path, shards, ticks):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    hb = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void k_refresh_score<true")]
    rows = rows[hb[shards]:] if len(hb) > shards else rows
    agg, cnt = collections.Counter(), collections.Counter()
    for r in rows:
        name = r["Kernel_Name"]
        name = name.split("(")[0] if not name.startswith("(") else name.split("::")[1].split("(")[0]
        agg[name] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cnt[name] += 1
    div = 1e6 * ticks * shards
    print(f"total {sum(agg.values()) / div:.3f} ms per tick per shard")
    for n, v in agg.most_common(18):
        print(f"  {n[-44:]:44s} {v / div:8.3f} ms  {cnt[n]:6d} dispatches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
