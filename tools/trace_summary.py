"""Summarise a rocprofv3 kernel trace (csv): per-kernel device time per tick.

usage: trace_summary.py TRACE.csv SHARDS [TICKS]

The first tick's dispatches are dropped (warm-up): the summary starts at the
(SHARDS+1)-th `k_refresh_score<true, ...>` dispatch, one per tick and shard.
The number of ticks kept is counted from those dispatches (TICKS, if given,
must agree).  Two columns: the time summed over the shards ("all shards"),
and that sum divided by SHARDS ("per shard", the mean shard -- the figure
bench.py's `kernel_ms_per_tick_shards` averages to under GSIM_GROUP_SERIAL=1).
With SHARDS = 1 the two are the same."""
import collections
import csv
import sys


def main(path, shards, ticks=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    hb = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void k_refresh_score<true")]
    rows = rows[hb[shards]:] if len(hb) > shards else rows
    kept = (len(hb) - shards) // shards if len(hb) > shards else 1
    if ticks is not None and ticks != kept:
        print(f"# note: {ticks} ticks requested, {kept} counted from the refresh dispatches; using {kept}")
    agg, cnt = collections.Counter(), collections.Counter()
    for r in rows:
        name = r["Kernel_Name"]
        name = name.split("(")[0] if not name.startswith("(") else name.split("::")[1].split("(")[0]
        agg[name] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cnt[name] += 1
    tot = sum(agg.values()) / (1e6 * kept)
    span = (max(int(r["End_Timestamp"]) for r in rows) - int(rows[0]["Start_Timestamp"])) / (1e6 * kept)
    print(f"{kept} ticks, {shards} shard(s): {tot:.3f} ms per tick all shards, {tot / shards:.3f} ms per tick per shard")
    print(f"  device span {span:.3f} ms per tick (first dispatch to last end; the gaps: {span - tot / shards:.3f} ms"
          f" with one shard), {len(rows) / kept:.1f} dispatches per tick")
    print(f"  {'kernel':44s} {'all shards':>10s} {'per shard':>10s}  dispatches")
    for n, v in agg.most_common(int(__import__('os').environ.get('TOPK', '20'))):
        ms = v / (1e6 * kept)
        print(f"  {n[-44:]:44s} {ms:10.3f} {ms / shards:10.3f}  {cnt[n]:6d}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else None)
