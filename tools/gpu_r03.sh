#!/bin/bash
# GPU: the -m gpu suite, then bench lines of the given configs (CPU baselines off).
#   CONFIGS="c3 c5" STEPS=10 tools/gpu_r03.sh TAG
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r03}"
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" "$OUT/pytest_gpu.log" | head -30; exit $rc; }
fi
for c in ${CONFIGS:-c3}; do
  timeout -k 10 "${BENCH_TIMEOUT:-400}" python -u bench.py --config "$c" --steps "${STEPS:-10}" --warmup "${WARMUP:-2}" \
    --no-cpu-baseline > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  rc=$?
  if [ $rc -ne 0 ]; then tail -20 "$OUT/bench_$c.err"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'hbm', d['config'].get('hbm_used_gb'), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/bench_$c.json" "$c"
done
