#!/bin/bash
# GPU (round 5): gossip marks exported in edge order and the holder import's
# g2l loads four words at a time -- shard parity, then serial K=8 A/B against
# the previous build.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05x"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_shard.py tests/test_configs.py tests/test_trace.py tests/test_gater.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest.log" | head -20; exit 1; }
tail -1 "$OUT/pytest.log"
LIBS="new:$L/libgsim.so prev:$L/libgsim_prev.so" ROUNDS=2 tools/gpu_ab_shards.sh r05x_s8
