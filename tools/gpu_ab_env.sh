#!/bin/bash
# GPU: A/B of one bench environment knob in one call.
#   VAR=GSIM_TM_SLOTS VALUES="0 1 2" CONFIGS="c3 c5" tools/gpu_ab_env.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-ab_env}"
mkdir -p "$OUT"
cd "$ROOT"
for c in ${CONFIGS:-c3}; do
  n=0
  for v in ${VALUES}; do
    n=$((n + 1))
    env "$VAR=$v" timeout -k 10 300 python bench.py --config "$c" --steps "${STEPS:-5}" --warmup 2 \
      --no-cpu-baseline > "$OUT/${c}_$n.json" 2> "$OUT/${c}_$n.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/${c}_$n.json" "$c $VAR=$v"
  done
done
