#!/bin/bash
# GPU (round 5): the shards' split commit over 2 / 4 / 8 topic groups and with
# 4-slot batches, serial K=8 C3 A/B, then the 8-group build's shard parity.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
LIBS="g4:$L/libgsim.so g8:$L/libgsim_sg8.so g2:$L/libgsim_sg2.so b4:$L/libgsim_sb4.so" ROUNDS=2 tools/gpu_ab_shards.sh r05y_s8 || exit 1
GSIM_LIB="$ROOT/$L/libgsim_sg8.so" timeout -k 10 400 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$ROOT/gpurun_out/r05y_s8/pytest_sg8.log" 2>&1; tail -1 "$ROOT/gpurun_out/r05y_s8/pytest_sg8.log"
