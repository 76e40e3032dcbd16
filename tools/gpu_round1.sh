#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
echo "== pytest -m gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
echo "== smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
echo "== bench"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
echo "== rocprofv3"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1
find "$OUT/prof" -name "*stats*" | head
echo "== done"
