#!/bin/bash
# GPU (round 6): c5's member-major IHAVE walk attributed (push / pull row walks, edges,
# hits, wave clocks per LP) with the -DGSIM_DIAG_IH build; then the c5 line of each
# build named in ARMS (libgsim_<arm>.so, "head" = libgsim.so), 10 warm-up ticks.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-r06ih}"
mkdir -p "$OUT"
L=go-libp2p-pubsub_amd
run_c5() {   # lib tag [env]
  env ${3:-} GSIM_LIB="$1" timeout -k 10 600 python -u bench.py --config c5 --steps "${STEPS:-3}" --warmup 10 \
    --no-cpu-baseline > "$OUT/$2.json" 2> "$OUT/$2.err" &
  local pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 30; echo "$2 running $(date +%T)"; done
  wait $pid || { echo "$2 rc=$?"; tail -5 "$OUT/$2.err"; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/$2.json" "$2"
}
if [ -z "${NO_DIAG:-}" ]; then
  run_c5 "$ROOT/$L/libgsim_ihdiag.so" diag GSIM_DIAG_IH=1 || exit 1
  grep ihave_counts "$OUT/diag.err"
fi
for arm in ${ARMS:-}; do          # an arm: a build name, or build:VAR=value (an environment setting)
  b="${arm%%:*}"; ev=""; [ "$b" != "$arm" ] && ev="${arm#*:}"
  lib="$ROOT/$L/libgsim_$b.so"; [ "$b" = head ] && lib="$ROOT/$L/libgsim.so"
  run_c5 "$lib" "c5_${arm//[:=]/_}" "$ev" || exit 1
done
echo "== done"
