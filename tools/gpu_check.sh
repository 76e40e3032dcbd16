#!/bin/bash
# GPU: the full -m gpu suite, then bench lines of the given configs.
#   CONFIGS="c3 c5" tools/gpu_check.sh TAG
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-check}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > "$OUT/pytest_gpu.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest_gpu.log" | head -30; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for c in ${CONFIGS:-c3}; do
  timeout -k 10 300 python bench.py --config "$c" --steps "${STEPS:-10}" --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), round(d['roofline']['frac'],4), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/bench_$c.json" "$c"
done
