#!/bin/bash
# GPU (round-5 final, part A): the whole -m gpu suite, smoke(), and the serial
# K=8 C3 line with its rocprofv3 kernel summary.  Part B is tools/gpu_measure.sh
# (the default C3 line, its kernel trace and the PMC passes behind traffic.json).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r05final}"
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { grep -E "FAILED|^E " "$OUT/pytest_gpu.log" | head -20; exit 1; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke fail"; tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
STEPS=5 tools/gpu_shard8.sh "${1:-r05final}_s8"
