#!/bin/bash
# GPU: k_send_tm grid size A/B (GSIM_TM_BLOCKS), one bench line per setting.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/tmb"
mkdir -p "$OUT"
cd "$ROOT"
for B in ${BLOCKS:-1024 512 2048 4096 1024}; do
  GSIM_TM_BLOCKS=$B timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_$B.log" 2>&1 || { tail -20 "$OUT/bench_$B.log"; exit 1; }
  echo "$B $(tail -1 "$OUT/bench_$B.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_tick']; print(round(d['ms_per_step'],2), round(k['send'],2), round(k['commit'],2))")"
done
