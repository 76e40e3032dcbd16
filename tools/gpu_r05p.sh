#!/bin/bash
# GPU (round 5): the split commit shared by topic (plain credits) -- shard
# parity, serial K=8 A/B against the dealt batches; C3 A/B of the refresh grid
# and the commit's slot batch.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05p"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest.log" | head -30; exit 1; }
tail -1 "$OUT/pytest.log"
LIBS="topic:$L/libgsim.so dealt:$L/libgsim_splitdealt.so" ROUNDS=2 tools/gpu_ab_shards.sh r05p_ab || exit 1
LIBS="base:$L/libgsim.so rg32k:$L/libgsim_rg32k.so rg128k:$L/libgsim_rg128k.so sb16:$L/libgsim_sb16.so sb4:$L/libgsim_sb4.so" \
  ROUNDS=2 STEPS=5 tools/gpu_ab_libs.sh r05p_c3
