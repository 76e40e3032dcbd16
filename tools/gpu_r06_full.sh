#!/bin/bash
# GPU (round 6): the bench-size parity tests (C3 at 1M for
# one tick, C4 at 125k over ticks 1-10; GSIM_FULL_SIZE=1, progress lines via -s),
# then the c5 line at 10M in steady state (10 warm-up ticks, 10 timed).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r06full}"
mkdir -p "$OUT"
if [ -z "${NO_FULL:-}" ]; then
  GSIM_FULL_SIZE=1 timeout -k 10 900 python -u -m pytest tests/test_fullsize.py -s -v --timeout 850 \
    --timeout-method thread 2>&1 | tee "$OUT/pytest_fullsize.log" | grep -E "fullsize|PASS|FAIL|Error|passed|failed"
  rc=${PIPESTATUS[0]}
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "${NO_C5:-}" ]; then
  timeout -k 10 900 python -u bench.py --config c5 --steps "${C5_STEPS:-10}" --warmup "${C5_WARMUP:-10}" ${C5_ARGS:-} \
    > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &
  pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 30; echo "c5 running $(date +%T)"; done
  wait $pid || { echo "c5 rc=$?"; tail -5 "$OUT/bench_c5.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/bench_c5.json"
fi
echo "== done"
