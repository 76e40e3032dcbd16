#!/bin/bash
# GPU: rocprofv3 kernel stats of one bench configuration (default c5).
set -euo pipefail
C="${1:-c5}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/prof_$C"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$C" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
tail -1 "$OUT/prof.log"
