#!/bin/bash
# GPU: topic-major block shares A/B on c5 (uniform per topic vs by subscribers),
# after the delivery parity tests.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-ab_blocks}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_configs.py tests/test_delivery.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1
for u in 1 0; do
  GSIM_TM_UNIFORM=$u timeout -k 10 300 python bench.py --config "${CONFIG:-c5}" --steps 5 --warmup 2 \
    --no-cpu-baseline > "$OUT/bench_u$u.json" 2> "$OUT/bench_u$u.err"
done
tail -2 "$OUT/pytest.log"
for u in 1 0; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items()})" "$OUT/bench_u$u.json" "uniform=$u"
done
