#!/bin/bash
# GPU session: parity tests, smoke, bench, rocprofv3 kernel stats, PMC traffic.
# usage: tools/gpu_session.sh <tag> [pytest-args...]
set -euo pipefail
TAG="${1:-run}"; shift || true
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
echo "== smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
echo "== bench"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
echo "== rocprofv3 kernel stats"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/prof.log" 2>&1
for K in refresh send; do
  if [ "$K" = refresh ]; then RE="k_refresh_score<true, true>"; else RE="k_send"; fi
  echo "== pmc FETCH_SIZE $K"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" -d "$OUT/pmc_fetch_$K" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_$K.log" 2>&1
  echo "== pmc WRITE_SIZE $K"
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" -d "$OUT/pmc_write_$K" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_$K.log" 2>&1
done
cd "$ROOT"
python3 tools/pmc_traffic.py c3 "k_refresh_score<true, ?true>" "$OUT/pmc_fetch_refresh" "$OUT/pmc_write_refresh" "$OUT/traffic.json" || true
python3 tools/pmc_traffic.py c3:send "k_send" "$OUT/pmc_fetch_send" "$OUT/pmc_write_send" "$OUT/traffic.json" || true
echo "== done"
