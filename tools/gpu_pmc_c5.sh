#!/bin/bash
# GPU: PMC passes over the c5 line's dominant kernels (TCC hit/miss and
# memory-side reads; TCP->TCC request mix), one rocprofv3 --pmc run each.
#   KRE="k_send_tm|k_ihave" tools/gpu_pmc_c5.sh TAG
set -uo pipefail
TAG="${1:-pmc_c5}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
KRE="${KRE:-k_send_tm|k_ihave|k_commit}"
export TMPDIR=/tmp
cd /tmp
pass() {
  local name="$1"; shift
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex "$KRE" -d "$OUT/pmc_$name" -o p \
    --output-format csv -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "$OUT/pmc_$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum && \
pass tcp TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum \
  || exit 1
cd "$ROOT"
python3 tools/pmc_parse.py "$OUT/pmc.json" "$OUT"/pmc_tcc "$OUT"/pmc_tcp > "$OUT/pmc.txt"
cat "$OUT/pmc.txt"
