#!/bin/bash
# GPU: parity tests, then the heartbeat A/B (packed 32-lane groups vs one observer per wave).
set -euo pipefail
TAG="${1:-hbab}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u tools/ab_deliver.py > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
tail -1 "$OUT/ab.log"
