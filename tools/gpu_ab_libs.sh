#!/bin/bash
# GPU: A/B/... of several builds of libgsim.so on one box, arms interleaved.
#   LIBS="base:go-libp2p-pubsub_amd/libgsim_a.so new:go-libp2p-pubsub_amd/libgsim.so" ROUNDS=2 CONFIGS="c3" tools/gpu_ab_libs.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-ab_libs}"
mkdir -p "$OUT"
cd "$ROOT"
for c in ${CONFIGS:-c3}; do
  for r in $(seq 1 "${ROUNDS:-2}"); do
    for arm in ${LIBS}; do
      name="${arm%%:*}"; lib="$ROOT/${arm#*:}"
      GSIM_LIB="$lib" timeout -k 10 300 python bench.py --config "$c" --steps "${STEPS:-5}" --warmup 2 \
        --no-cpu-baseline > "$OUT/${c}_${name}_$r.json" 2> "$OUT/${c}_${name}_$r.err"
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/${c}_${name}_$r.json" "$c $name $r"
    done
  done
done
