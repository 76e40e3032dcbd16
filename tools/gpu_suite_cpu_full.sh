#!/bin/bash
# GPU: the -m gpu suite (optionally -k), then -- unless NO_CPU_FULL -- the
# C oracle on the full 1M-peer C3 network on the box's own host cores
# (bench.py --cpu-full, all-core leg; VERDICT r3 "Next" #9).  Outputs under
# gpurun_out/TAG.  The CPU leg prints a progress line every 30 s (it runs
# minutes without output of its own).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-suite}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "^E |FAILED|passed|failed" "$OUT/pytest_gpu.log" | head -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
[ -n "${NO_CPU_FULL:-}" ] && exit 0
nproc > "$OUT/nproc.txt"
echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset} nproc=$(nproc)"
GSIM_CPU_LEGS=all timeout -k 10 900 python -u bench.py --cpu-full --config c3 > "$OUT/cpu_full_c3.json" 2> "$OUT/cpu_full_c3.err" &
pid=$!
while kill -0 $pid 2>/dev/null; do
  sleep 30
  echo "cpu-full running $(date +%T)"
done
wait $pid
rc=$?
cat "$OUT/cpu_full_c3.json"
exit $rc
