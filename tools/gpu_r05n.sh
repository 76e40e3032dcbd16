#!/bin/bash
# GPU (round-5 final, part B): the list-capacity and invalid-plane parity
# tests, the HEAD measurement set (tools/gpu_measure.sh: C3 line, kernel
# trace, PMC passes), then the c5 line on the round-4 window.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r05n"
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_verdicts.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest.log" | head -30; exit 1; }
tail -1 "$OUT/pytest.log"
tools/gpu_measure.sh r05fm || exit 1
timeout -k 10 600 python -u bench.py --config c5 --steps 4 --warmup 2 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { echo "c5 fail"; tail "$OUT/bench_c5.err"; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', round(d['ms_per_step'],2), {x: round(v,1) for x,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/bench_c5.json"
