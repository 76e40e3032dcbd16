#!/bin/bash
# GPU (round 5): the single engine's commit over 4 / 8 topic groups (as the
# shards' split commit) against the wave-per-word scan on C3, and the delivery
# parity of the 4-group build.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05t"
mkdir -p "$OUT"
GSIM_LIB="$ROOT/$L/libgsim_ss.so" timeout -k 10 400 python -u -m pytest tests/test_delivery.py tests/test_verdicts.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_ss.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest_ss.log" | head -20; exit 1; }
tail -1 "$OUT/pytest_ss.log"
LIBS="base:$L/libgsim.so ss:$L/libgsim_ss.so ss8:$L/libgsim_ss8.so" ROUNDS=2 STEPS=5 tools/gpu_ab_libs.sh r05t_c3
