#!/bin/bash
# GPU: full parity suite, then the c5 bench line (churn every tick) and C3.
set -euo pipefail
TAG="${1:-churn}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for C in c5 c3; do
  timeout -k 10 400 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench_$C.log" 2>&1 || { tail -20 "$OUT/bench_$C.log"; exit 1; }
  tail -1 "$OUT/bench_$C.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$C', round(d['ms_per_step'],2), d['kernel_ms_per_tick'])"
done
