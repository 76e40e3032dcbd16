#!/bin/bash
# GPU (round 5): A/B of the shard push-walk / bit-apply builds on the serial
# K=8 C3 line, k_send_tm's phase clocks (diagnostic build), then the c4 / c2 /
# c5 bench lines at HEAD.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05h"
mkdir -p "$OUT"
GSIM_DIAG_PHASE=1 GSIM_LIB="$ROOT/$L/libgsim_diagph.so" timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
  --no-cpu-baseline > "$OUT/diag.json" 2> "$OUT/diag.err" || { echo "diag fail"; tail "$OUT/diag.err"; exit 1; }
grep send_phase "$OUT/diag.err"
python3 -c "import json; d=json.loads(open('$OUT/diag.json').read().strip().splitlines()[-1]); print('diag', round(d['ms_per_step'],2), d['kernel_ms_per_tick']['send'])"
LIBS="base:$L/libgsim.so p512w6:$L/libgsim_p512w6.so p512w4:$L/libgsim_p512w4.so xbw6:$L/libgsim_xbw6.so xbp4:$L/libgsim_xbp4.so" \
  ROUNDS=2 tools/gpu_ab_shards.sh r05h_ab || exit 1
CONFIGS="c4 c2 c5" tools/gpu_configs.sh r05_cfg
