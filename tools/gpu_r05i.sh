#!/bin/bash
# GPU (round 5): send ranges down to one chunk -- c2 / c4 / C3 lines, the
# delivery parity tests, and c5 (5 timed ticks: its 96-slot sub-rings hold
# ~20 ticks of publications).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r05i"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_delivery.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest.log" | head -30; exit 1; }
tail -1 "$OUT/pytest.log"
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_tick']; print(sys.argv[2], round(d['ms_per_step'],3), {x: round(v,3) for x,v in k.items() if v > 0.01})" "$1" "$2"; }
for C in c2 c4; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" || { echo "$C fail"; tail "$OUT/bench_$C.err"; exit 1; }
  line "$OUT/bench_$C.json" $C
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || { echo "c3 fail"; exit 1; }
line "$OUT/bench_c3.json" c3
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 2 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { echo "c5 fail"; tail "$OUT/bench_c5.err"; exit 1; }
line "$OUT/bench_c5.json" c5
