#!/bin/bash
# GPU session: parity tests + in-process kernel A/B + bench.
set -euo pipefail
TAG="${1:-ab}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
echo "== A/B"
timeout -k 10 400 python -u tools/ab_kernels.py --diag > "$OUT/ab.log" 2>&1
tail -1 "$OUT/ab.log"
echo "== bench"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
