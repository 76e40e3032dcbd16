#!/bin/bash
# GPU (round 6): the heartbeat's reads attributed with builds
# whose results are unchanged.  Arms: hbbase (every gather), hbsub (no sub[col]
# gather when every peer joined every topic), head (that + no invalid-plane
# loads in the live re-score while the refresh's flag says zero).  Per arm: the
# C3 line (kernel ms) and one PMC pass on k_heartbeat<32> (TCC_EA0_RDREQ,
# TCC_HIT / MISS); the hbdiag build counts re-scores / Grafts / Prunes / backoff loads.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r06hb}"
mkdir -p "$OUT"
L=go-libp2p-pubsub_amd
GSIM_LIB="$ROOT/$L/libgsim_hbdiag.so" GSIM_DIAG_HB=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 \
  --no-cpu-baseline > "$OUT/diag.json" 2> "$OUT/diag.err" || { echo "diag rc=$?"; tail -5 "$OUT/diag.err"; exit 1; }
grep heartbeat_counts "$OUT/diag.err"
GSIM_LIB="$ROOT/$L/libgsim_phase.so" GSIM_DIAG_PHASE=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 \
  --no-cpu-baseline > "$OUT/phase.json" 2> "$OUT/phase.err" || { echo "phase rc=$?"; tail -5 "$OUT/phase.err"; exit 1; }
grep send_phase "$OUT/phase.err"
for r in 1 2; do
  for arm in hbbase hbsub head; do
    lib="$ROOT/$L/libgsim_$arm.so"; [ "$arm" = head ] && lib="$ROOT/$L/libgsim.so"
    GSIM_LIB="$lib" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      > "$OUT/c3_${arm}_$r.json" 2> "$OUT/c3_${arm}_$r.err" || { echo "bench $arm rc=$?"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/c3_${arm}_$r.json" "$arm $r"
  done
done
export TMPDIR=/tmp
for arm in hbbase hbsub head; do
  lib="$ROOT/$L/libgsim_$arm.so"; [ "$arm" = head ] && lib="$ROOT/$L/libgsim.so"
  (cd /tmp && GSIM_LIB="$lib" timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum \
    --kernel-include-regex "k_heartbeat<32>" -d "$OUT/pmc_$arm" -o p --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$arm.log" 2>&1) || { echo "pmc $arm failed"; exit 1; }
  echo "pmc $arm ok"
done
echo "== done"
