#!/bin/bash
# GPU (round 5): C3 line at HEAD and with the diagnostic cheap selection keys
# (the heartbeat's Philox price), arms interleaved; then the serial 8-shard
# C3 line and its rocprof kernel summary (tools/gpu_shard8.sh).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r05e}"
mkdir -p "$OUT"
cd "$ROOT"
P=go-libp2p-pubsub_amd
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_tick']; print(sys.argv[2], round(d['ms_per_step'],2), {x: round(v,2) for x,v in k.items() if v > 0.05})" "$1" "$2"; }
for r in 1 2; do
  for arm in new cheapkey; do
    lib="$ROOT/$P/libgsim_$arm.so"; [ "$arm" = new ] && lib="$ROOT/$P/libgsim.so"
    GSIM_LIB="$lib" timeout -k 10 240 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > "$OUT/b_${arm}_$r.json" 2> "$OUT/b_${arm}_$r.err" || { echo "bench $arm fail"; tail "$OUT/b_${arm}_$r.err"; exit 1; }
    line "$OUT/b_${arm}_$r.json" "$arm $r"
  done
done
STEPS=3 tools/gpu_shard8.sh "${1:-r05e}_s8"
