#!/bin/bash
# GPU: the sharded-path tests, then per-shard kernel time of the in-process
# K-shard C3 run (GSIM_GROUP_SERIAL=1: each shard alone on the device), push
# against pull.
#   TESTS="tests/test_shard.py" KS="8" MODES="0 1" tools/gpu_shards.sh TAG
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-shards}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS} -m gpu -x -v --timeout 600 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" "$OUT/pytest_gpu.log" | head -30; exit $rc; }
fi
for k in ${KS:-8}; do
  for pull in ${MODES:-0 1}; do
    GSIM_GROUP_SERIAL=1 GSIM_SHARD_PULL=$pull timeout -k 10 400 python bench.py --config "${CONFIG:-c3}" --shards "$k" \
      --steps "${STEPS:-3}" --warmup 1 --no-cpu-baseline > "$OUT/k${k}_pull${pull}.json" 2> "$OUT/k${k}_pull${pull}.err"
    rc=$?
    [ $rc -ne 0 ] && { tail -20 "$OUT/k${k}_pull${pull}.err"; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), d['kernel_ms_per_tick_shards'], {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/k${k}_pull${pull}.json" "K=$k pull=$pull"
  done
done
