#!/bin/bash
# GPU: the sharded parity tests, then the serial 8-shard C3 line with its
# kernel trace (tools/gpu_shard8.sh).   tools/gpu_shardcheck.sh TAG
set -uo pipefail
TAG="${1:-shardcheck}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p "gpurun_out/$TAG"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "${PYTEST_K:-shard or latency}" > "gpurun_out/$TAG/pytest_gpu.log" 2>&1
rc=$?
grep -E "^E |FAILED|passed|failed" "gpurun_out/$TAG/pytest_gpu.log" | head -20
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_shard8.sh "${TAG}8"
