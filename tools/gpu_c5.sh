#!/bin/bash
# GPU: optional -m gpu tests (PYTEST_K), then the c5 line (10M peers) and a
# rocprofv3 kernel trace of it, summarised per kernel per tick.
#   PYTEST_K="gpu_score" tools/gpu_c5.sh TAG
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-c5}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  grep -E "^E |FAILED|passed|failed" "$OUT/pytest_gpu.log" | head -20
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 700 python -u bench.py --config c5 --steps "${STEPS:-4}" --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
  > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench_c5.err"; exit 1; }
python3 tools/bench_summary.py "$OUT/bench_c5.json"
[ -n "${NO_PROF:-}" ] && exit 0
export TMPDIR=/tmp
cd /tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o s \
  -- python3 "$ROOT/bench.py" --config c5 --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof.json" 2> "$OUT/prof.err" \
  || { echo "prof rc=$?"; tail -20 "$OUT/prof.err"; exit 1; }
python3 "$ROOT/tools/trace_summary.py" "$OUT/prof/s_kernel_trace.csv" 1 > "$OUT/prof_summary.txt"; head -26 "$OUT/prof_summary.txt"
