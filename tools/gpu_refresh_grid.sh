#!/bin/bash
# GPU: refresh grid-size A/B (GSIM_REFRESH_GRID_CAP), one bench line per setting.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/rg"
mkdir -p "$OUT"
cd "$ROOT"
for C in ${CAPS:-16384 4096 8192 32768 131072 16384}; do
  GSIM_REFRESH_GRID_CAP=$C timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_$C.log" 2>&1 || { tail -20 "$OUT/bench_$C.log"; exit 1; }
  echo "$C $(tail -1 "$OUT/bench_$C.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_tick']; print(round(d['ms_per_step'],2), round(k['refresh_score'],2))")"
done
