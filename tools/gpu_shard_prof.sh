#!/bin/bash
# GPU: kernel trace of the in-process sharded group run serially (each shard
# alone on the device), summarised per kernel per tick per shard.
set -euo pipefail
TAG="${1:-shprof}"
S="${SHARDS:-8}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp GSIM_GROUP_SERIAL=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof$S" -o s -- \
  python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --shards "$S" > "$OUT/prof$S.log" 2>&1
python3 "$ROOT/tools/trace_summary.py" "$OUT/prof$S/s_kernel_trace.csv" "$S" 3
