#!/bin/bash
# GPU (round 5): c5 at 10M on the round-4 window (4 timed ticks after 2), the
# claim / forwarder list capacity (GSIM_CLIST_MULT x N entries) 2 / 4 / 8.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05l"
mkdir -p "$OUT"
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_tick']; print(sys.argv[2], round(d['ms_per_step'],2), {x: round(v,1) for x,v in k.items() if v > 0.05}, d['config']['hbm_used_gb'])" "$1" "$2"; }
for arm in cl4:$L/libgsim_cl4.so cl8:$L/libgsim_cl8.so base:$L/libgsim.so; do
  name="${arm%%:*}"; lib="$ROOT/${arm#*:}"
  GSIM_LIB="$lib" timeout -k 10 500 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/c5_$name.json" 2> "$OUT/c5_$name.err" || { echo "c5 $name fail"; tail "$OUT/c5_$name.err"; exit 1; }
  line "$OUT/c5_$name.json" "c5 $name"
done
