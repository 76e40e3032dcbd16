#!/bin/bash
# GPU: A/B of libgsim builds on the serial K-shard C3 line (per-shard kernel
# ms per tick, HIP events), arms interleaved on one box.
#   LIBS="base:go-libp2p-pubsub_amd/libgsim.so p512:go-libp2p-pubsub_amd/libgsim_p512.so" ROUNDS=2 tools/gpu_ab_shards.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-ab_shards}"
mkdir -p "$OUT"
cd "$ROOT"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for arm in ${LIBS}; do
    name="${arm%%:*}"; lib="$ROOT/${arm#*:}"
    GSIM_GROUP_SERIAL=1 GSIM_LIB="$lib" timeout -k 10 300 python bench.py --shards "${K:-8}" --steps "${STEPS:-3}" --warmup 2 \
      --no-cpu-baseline > "$OUT/s_${name}_$r.json" 2> "$OUT/s_${name}_$r.err"
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s=d['kernel_ms_per_tick_shards']
print(sys.argv[2], round(d['ms_per_step'],2), 'per-shard', s, 'mean', round(sum(s)/len(s),2), 'max', max(s))
print('   ', {a: round(b,2) for a,b in d['kernel_ms_per_tick'].items() if b > 0.05})" "$OUT/s_${name}_$r.json" "$name $r"
  done
done
