#!/bin/bash
# GPU: kernel trace of one bench configuration (single engine), summarised per
# kernel per tick over the timed ticks.
set -euo pipefail
TAG="${1:-prof}"
CFG="${CONFIG:-c3}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$CFG" -o s -- \
  python3 "$ROOT/bench.py" --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$CFG.log" 2>&1
python3 "$ROOT/tools/trace_summary.py" "$OUT/$CFG/s_kernel_trace.csv" 1 3
