#!/bin/bash
# GPU (round 5): the commit with every lastput / credit load of a slot batch
# issued before its stores -- delivery / verdict / shard / c5-shape parity, then
# C3 and serial K=8 A/B against the one-claim-at-a-time commit.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05u"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_delivery.py tests/test_verdicts.py tests/test_shard.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest.log" | head -20; exit 1; }
tail -1 "$OUT/pytest.log"
LIBS="batched:$L/libgsim.so serial:$L/libgsim_cb0.so" ROUNDS=2 STEPS=5 tools/gpu_ab_libs.sh r05u_c3 || exit 1
LIBS="batched:$L/libgsim.so serial:$L/libgsim_cb0.so" ROUNDS=1 tools/gpu_ab_shards.sh r05u_s8
