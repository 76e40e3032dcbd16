#!/bin/bash
# GPU: A/B of the topic-major walk (gsim_set_kernel_variant(h, 4, v)) on the
# single engine and a sharded group: per-tick time and kernel classes.
set -euo pipefail
TAG="${1:-walk}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for S in ${SHARDS:-1 2}; do
  for V in ${WALKS:-1 2}; do
    echo "== shards $S walk $V"
    GSIM_GROUP_SERIAL=${SERIAL:-0} GSIM_TM_WALK=$V timeout -k 10 400 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --shards $S > "$OUT/bench_s${S}_w$V.log" 2>&1 || { tail -30 "$OUT/bench_s${S}_w$V.log"; exit 1; }
    tail -1 "$OUT/bench_s${S}_w$V.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), d.get('kernel_ms_per_tick_shards'), {k: round(v,2) for k, v in d['kernel_ms_per_tick'].items() if v})"
  done
done
