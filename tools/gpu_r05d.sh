#!/bin/bash
# GPU (round 5): parity of the list-driven send and the batched bit apply,
# then c5 at 10M (list vs scan) and the serial 8-shard C3 line + profile.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r05d}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_configs.py tests/test_subscriptions.py tests/test_shard.py tests/test_delivery.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest.log" | head -30; exit 1; }
tail -1 "$OUT/pytest.log"
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_tick']; print(sys.argv[2], round(d['ms_per_step'],2), {x: round(v,2) for x,v in k.items() if v > 0.05}, d.get('shard_kernel_ms_per_tick'))" "$1" "$2"; }
for arm in list scan; do
  ev=""; [ "$arm" = scan ] && ev="GSIM_FLIST_OFF=1"
  env $ev timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c5_$arm.json" 2> "$OUT/c5_$arm.err" || { echo "c5 $arm fail"; tail "$OUT/c5_$arm.err"; exit 1; }
  line "$OUT/c5_$arm.json" "c5 $arm"
done
for arm in fast generic; do
  ev=""; [ "$arm" = generic ] && ev="GSIM_XB_GENERIC=1"
  env GSIM_GROUP_SERIAL=1 $ev timeout -k 10 400 python bench.py --shards 8 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/s8_$arm.json" 2> "$OUT/s8_$arm.err" || { echo "s8 $arm fail"; tail "$OUT/s8_$arm.err"; exit 1; }
  line "$OUT/s8_$arm.json" "s8 $arm"
done
