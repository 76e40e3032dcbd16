#!/bin/bash
# GPU: one test file, an env A/B on given configs, and a kernel profile of one config.
#   TESTS=tests/test_wire.py VAR=GSIM_TM_XCD VALUES="0 1" CONFIGS="c3" PROF=c5 tools/gpu_r03b.sh TAG
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03b}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS} -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" "$OUT/pytest_gpu.log" | head -30; exit $rc; }
fi
if [ -n "${VAR:-}" ]; then
  STEPS="${STEPS:-5}" VAR="$VAR" VALUES="$VALUES" CONFIGS="${CONFIGS:-c3}" tools/gpu_ab_env.sh "$TAG/ab" || exit $?
fi
if [ -n "${PROF:-}" ]; then
  CONFIG="$PROF" tools/gpu_prof_config.sh "$TAG/prof" > "$OUT/prof_$PROF.txt" 2>&1 || { tail -20 "$OUT/prof_$PROF.txt"; exit 1; }
  head -40 "$OUT/prof_$PROF.txt"
fi
