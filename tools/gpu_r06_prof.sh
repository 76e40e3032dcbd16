#!/bin/bash
# GPU (round 6): kernel traces of c2 / c4 (one-call ticks, launch gaps) and of
# c5 in steady state (10 warm-up ticks), summarised per tick.
set -uo pipefail
TAG="${1:-r06prof}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for CFG in ${CONFIGS:-c2 c4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$CFG" -o s -- \
    python3 "$ROOT/bench.py" --config "$CFG" --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/$CFG.json" 2> "$OUT/$CFG.err" || exit $?
  TOPK=40 python3 "$ROOT/tools/trace_summary.py" "$OUT/$CFG/s_kernel_trace.csv" 1 | tee "$OUT/${CFG}_summary.txt"
done
if [ -n "${C5:-}" ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5" -o s -- \
    python3 "$ROOT/bench.py" --config c5 --steps ${C5_STEPS:-3} --warmup 10 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 30; echo "c5 running $(date +%T)"; done
  wait $pid || exit 1
  python3 - "$OUT/c5/s_kernel_trace.csv" "${C5_STEPS:-3}" > "$OUT/c5_summary.txt" <<'PY'
import csv, collections, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
hb = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void k_refresh_score<true")]
K = int(sys.argv[2])
rows = rows[hb[-K]:]          # the timed ticks
agg, cnt = collections.Counter(), collections.Counter()
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    agg[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"]); cnt[n] += 1
print(f"c5, {K} timed ticks after 10 warm-up: {sum(agg.values()) / (K * 1e6):.2f} ms per tick")
for n, v in agg.most_common(40):
    print(f"  {n[-70:]:70s} {v / (K * 1e6):9.3f}  {cnt[n]:6d}")
PY
  head -30 "$OUT/c5_summary.txt"
fi
echo "== done"
