#!/bin/bash
# GPU (round-5 final): c5 at 10M on the round-4 window with the CPU baseline,
# and c5's shape at 2M on one engine and 8 serial shards, at HEAD.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r05r"
mkdir -p "$OUT"
timeout -k 10 600 python -u bench.py --config c5 --steps 4 --warmup 2 > "$OUT/c5.json" 2> "$OUT/c5.err" || { echo "c5 fail"; tail "$OUT/c5.err"; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', round(d['ms_per_step'],2), {x: round(v,1) for x,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/c5.json"
tools/gpu_r05o.sh
L=go-libp2p-pubsub_amd
LIBS="base:$L/libgsim.so fc16:$L/libgsim_fc16.so" ROUNDS=2 STEPS=5 tools/gpu_ab_libs.sh r05r_c3
