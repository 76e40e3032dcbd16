#!/bin/bash
# GPU (round 6): the -m gpu suite, smoke(), and short bench lines of c3 / c2 / c4
# (each step under its own time limit; the first failure ends the script).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r06}"
mkdir -p "$OUT"
if [ -z "${NO_SUITE:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  grep -E "^E |FAILED|passed|failed" "$OUT/pytest_gpu.log" | head -30
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
for c in ${CONFIGS:-c3 c2 c4}; do
  timeout -k 10 300 python -u bench.py --config "$c" --steps "${STEPS:-10}" --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { echo "bench $c rc=$?"; tail -5 "$OUT/bench_$c.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernel_ms_per_tick'].items() if v > 0.01})" "$OUT/bench_$c.json" "$c"
done
echo "== done"
