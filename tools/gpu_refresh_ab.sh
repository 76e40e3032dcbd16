#!/bin/bash
# GPU: refresh+score parity for every variant, then in-process A/B of the variants
# (tools/ab_kernels.py) and one bench line per GSIM_SCORE_KERNEL setting.
set -euo pipefail
TAG="${1:-rab}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_score.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_score.log" 2>&1 || { tail -30 "$OUT/pytest_score.log"; exit 1; }
tail -1 "$OUT/pytest_score.log"
timeout -k 10 400 python -u tools/ab_kernels.py --rounds 5 --iters 5 > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
tail -1 "$OUT/ab.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['refresh_ms']))"
for K in thread pipe thread pipe; do
  GSIM_SCORE_KERNEL=$K timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_$K.log" 2>&1 || { tail -20 "$OUT/bench_$K.log"; exit 1; }
  echo "$K $(tail -1 "$OUT/bench_$K.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_tick']; print(round(d['ms_per_step'],2), round(k['refresh_score'],2))")"
done
