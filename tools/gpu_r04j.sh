#!/bin/bash
# GPU: the c5 line (no profile), the parity tests of the hub / IHAVE / sharded
# copy-bit changes, then the serial 8-shard C3 line with its kernel trace.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/r04j
NO_PROF=1 bash tools/gpu_c5.sh r04j || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "shard or c5_combined or hub_rows or px or gossip or topic_slots" > gpurun_out/r04j/pytest_gpu.log 2>&1
rc=$?
grep -E "^E |FAILED|passed|failed" gpurun_out/r04j/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_shard8.sh r04j8
