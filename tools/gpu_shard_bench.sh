#!/bin/bash
# GPU: bench lines for the single engine and the in-process sharded group on one GPU.
set -euo pipefail
TAG="${1:-shb}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for S in ${SHARDS:-1 2 4}; do
  echo "== shards $S"
  timeout -k 10 400 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --shards $S > "$OUT/bench_s$S.log" 2>&1 || { tail -30 "$OUT/bench_s$S.log"; exit 1; }
  tail -1 "$OUT/bench_s$S.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), d['msg_edge_deliveries_per_sec'], {k: round(v,2) for k, v in d['kernel_ms_per_tick'].items()})"
done
