#!/bin/bash
# GPU (round 5): shard push-walk ranges / split-commit A/B (serial K=8 C3), the
# split-commit variant's shard parity, then c5 list vs scan on the round-4
# window (tools/gpu_r05j.sh).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05k"
mkdir -p "$OUT"
GSIM_LIB="$ROOT/$L/libgsim_sw4.so" timeout -k 10 400 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_sw4.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest_sw4.log" | head -30; exit 1; }
tail -1 "$OUT/pytest_sw4.log"
LIBS="base:$L/libgsim.so pr2:$L/libgsim_pr2.so pr4:$L/libgsim_pr4.so sw4:$L/libgsim_sw4.so sw4g2:$L/libgsim_sw4g2.so" \
  ROUNDS=2 tools/gpu_ab_shards.sh r05k_ab || exit 1
tools/gpu_r05j.sh
