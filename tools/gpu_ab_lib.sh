#!/bin/bash
# GPU: A/B of two builds of libgsim.so on one box, arms interleaved.
#   LIB_A=go-libp2p-pubsub_amd/libgsim_a.so ROUNDS=3 CONFIGS="c3" tools/gpu_ab_lib.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-ab_lib}"
mkdir -p "$OUT"
cd "$ROOT"
for c in ${CONFIGS:-c3}; do
  for r in $(seq 1 "${ROUNDS:-3}"); do
    for arm in a b; do
      if [ "$arm" = a ]; then lib="$ROOT/${LIB_A}"; else lib="$ROOT/go-libp2p-pubsub_amd/libgsim.so"; fi
      GSIM_LIB="$lib" timeout -k 10 300 python bench.py --config "$c" --steps "${STEPS:-5}" --warmup 2 \
        --no-cpu-baseline > "$OUT/${c}_${arm}_$r.json" 2> "$OUT/${c}_${arm}_$r.err"
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/${c}_${arm}_$r.json" "$c $arm $r"
    done
  done
done
