#!/bin/bash
# GPU: A/B of environment knobs on one build, arms interleaved.
#   ENVS="base: w16:GSIM_IHAVE_W=16 w64:GSIM_IHAVE_W=64" ROUNDS=2 CONFIGS="c3" tools/gpu_ab_envs.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-ab_env}"
mkdir -p "$OUT"
cd "$ROOT"
for c in ${CONFIGS:-c3}; do
  for r in $(seq 1 "${ROUNDS:-2}"); do
    for arm in ${ENVS}; do
      name="${arm%%:*}"; ev="${arm#*:}"
      env $ev timeout -k 10 300 python bench.py --config "$c" --steps "${STEPS:-5}" --warmup 2 \
        --no-cpu-baseline > "$OUT/${c}_${name}_$r.json" 2> "$OUT/${c}_${name}_$r.err"
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/${c}_${name}_$r.json" "$c $name $r"
    done
  done
done
