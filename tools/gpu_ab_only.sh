#!/bin/bash
# Ablation timing only (tools/ab_deliver.py).
set -euo pipefail
TAG="${1:-ab}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 500 python -u tools/ab_deliver.py --rounds 2 --ticks 2 > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
tail -1 "$OUT/ab.log"
