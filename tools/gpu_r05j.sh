#!/bin/bash
# GPU (round 5): c5 at 10M, list-driven send against the scan, on the round-4
# final line's window (4 timed ticks after 2 warm-up ticks), one box.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r05j"
mkdir -p "$OUT"
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_tick']; print(sys.argv[2], round(d['ms_per_step'],2), {x: round(v,1) for x,v in k.items() if v > 0.05})" "$1" "$2"; }
for arm in list scan; do
  ev=""; [ "$arm" = scan ] && ev="GSIM_FLIST_OFF=1"
  env $ev timeout -k 10 500 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/c5_$arm.json" 2> "$OUT/c5_$arm.err" || { echo "c5 $arm fail"; tail "$OUT/c5_$arm.err"; exit 1; }
  line "$OUT/c5_$arm.json" "c5 $arm"
done
