#!/bin/bash
# GPU: the HEAD measurement set behind bench.py's roofline fields (VERDICT r3
# "Next" #1).  Outputs under gpurun_out/TAG:
#   bench.json        the default C3 line (CPU baseline on)
#   prof/             rocprofv3 --kernel-trace --stats of the same command
#   pmc_*             one rocprofv3 --pmc pass each (kernel-trace only):
#                     FETCH_SIZE; WRITE_SIZE; TCC hit / miss / memory-side
#                     reads; TCP->TCC request mix; the heartbeat's SQ counts
#   pmc.json          per-kernel per-launch means of every pass (pmc_parse.py)
set -uo pipefail
TAG="${1:-measure}"
STEPS="${STEPS:-20}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 600 python -u bench.py --steps "$STEPS" --warmup 3 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
  python3 tools/bench_summary.py "$OUT/bench.json"
fi
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o s \
  -- python3 "$ROOT/bench.py" --steps "$STEPS" --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof.json" 2> "$OUT/prof.err" \
  || { echo "prof rc=$?"; tail -20 "$OUT/prof.err"; exit 1; }
python3 "$ROOT/tools/trace_summary.py" "$OUT/prof/s_kernel_trace.csv" 1 > "$OUT/prof_summary.txt"; head -14 "$OUT/prof_summary.txt"
KRE="${KRE:-k_refresh_score<true, true>|k_send_tm|k_commit|k_heartbeat<32>}"
pass() {
  local name="$1"; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex "$KRE" -d "$OUT/pmc_$name" -o p \
    --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} \
    > "$OUT/pmc_$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE && \
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum && \
pass tcp TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum && \
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
  || exit 1
cd "$ROOT"
python3 tools/pmc_parse.py "$OUT/pmc.json" "$OUT"/pmc_fetch "$OUT"/pmc_write "$OUT"/pmc_tcc "$OUT"/pmc_tcp "$OUT"/pmc_sq > "$OUT/pmc.txt"
cat "$OUT/pmc.txt"
echo "== done"
