#!/bin/bash
# GPU: c5 bench lines for libgsim variants (GSIM_LIB), after a parity check of
# the default build.   VARIANTS="tb512 tb256" tools/gpu_ab_c5.sh TAG
set -uo pipefail
TAG="${1:-abc5}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  grep -E "^E |FAILED|passed|failed" "$OUT/pytest_gpu.log" | head -20
  [ $rc -ne 0 ] && exit $rc
fi
for v in default ${VARIANTS:-}; do
  if [ "$v" = default ]; then unset GSIM_LIB; else export GSIM_LIB="$ROOT/go-libp2p-pubsub_amd/libgsim_$v.so"; fi
  timeout -k 10 500 python -u bench.py --config "${CONFIG:-c5}" --steps "${STEPS:-4}" --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || { echo "bench $v rc=$?"; tail -5 "$OUT/bench_$v.err"; exit 1; }
  echo "== $v"; python3 tools/bench_summary.py "$OUT/bench_$v.json" | grep -v "^c5:"
done
