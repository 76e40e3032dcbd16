#!/bin/bash
# GPU: sharded parity after the holder-bits change, the serial 8-shard C3
# line with its kernel trace, then the c5 line with its kernel trace.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/r04k
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "shard or latency or px or c5_combined or hub_rows" > gpurun_out/r04k/pytest_gpu.log 2>&1
rc=$?
grep -E "^E |FAILED|passed|failed" gpurun_out/r04k/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_shard8.sh r04k8 || exit 1
bash tools/gpu_c5.sh r04kc5
