#!/bin/bash
# GPU: the in-process K-shard group on one GPU, each shard's work serialised
# (GSIM_GROUP_SERIAL=1: per-shard kernel times as if each shard had the device
# to itself) -- the bench line (kernel_ms_per_tick_shards) and a rocprofv3
# kernel trace summarised per kernel, summed over the shards and per shard.
#   SHARDS=8 tools/gpu_shard8.sh TAG
set -uo pipefail
TAG="${1:-sh8}"
S="${SHARDS:-8}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export GSIM_GROUP_SERIAL=1
timeout -k 10 500 python -u bench.py --steps "${STEPS:-5}" --warmup 2 --no-cpu-baseline --shards "$S" ${BENCH_ARGS:-} \
  > "$OUT/bench_s$S.json" 2> "$OUT/bench_s$S.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench_s$S.err"; exit 1; }
python3 - "$OUT/bench_s$S.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["kernel_ms_per_tick_shards"]
print("wall", round(d["ms_per_step"], 2), "ms/tick; per-shard kernel ms/tick", s, "mean", round(sum(s) / len(s), 2),
      "max", max(s))
print({k: round(v, 2) for k, v in d["kernel_ms_per_tick"].items() if v > 0.05})
PY
[ -n "${NO_PROF:-}" ] && exit 0
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o s \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --shards "$S" ${BENCH_ARGS:-} > "$OUT/prof.json" 2> "$OUT/prof.err" \
  || { echo "prof rc=$?"; tail -20 "$OUT/prof.err"; exit 1; }
python3 "$ROOT/tools/trace_summary.py" "$OUT/prof/s_kernel_trace.csv" "$S" > "$OUT/prof_summary.txt"; head -30 "$OUT/prof_summary.txt"
