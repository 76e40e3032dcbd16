#!/bin/bash
# GPU: bench lines for the BASELINE configurations beside C3 (c2, c4, c5).
set -euo pipefail
TAG="${1:-cfg}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for C in ${CONFIGS:-c4 c2 c5}; do
  echo "== $C"
  timeout -k 10 400 python -u bench.py --config $C --steps 20 --warmup 3 > "$OUT/bench_$C.log" 2>&1 || { tail -20 "$OUT/bench_$C.log"; exit 1; }
  tail -1 "$OUT/bench_$C.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['msg_edge_deliveries_per_sec'], d['kernel_ms_per_tick'])"
done
