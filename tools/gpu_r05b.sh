#!/bin/bash
# GPU (round 5): heartbeat / delivery parity, then C3 lines with the delivery
# kernel from launch order (default) and from XCD work queues (GSIM_TM_XCD).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r05b}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_heartbeat.py tests/test_delivery.py tests/test_gossip.py tests/test_configs.py tests/test_shard.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest.log" | head -30; exit 1; }
tail -1 "$OUT/pytest.log"
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_tick']; print(sys.argv[2], round(d['ms_per_step'],2), {x: round(v,2) for x,v in k.items() if v > 0.05})" "$1" "$2"; }
for r in 1 2; do
  for v in ${XCD_ARMS:-0 1}; do
    GSIM_TM_XCD=$v timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/xcd${v}_$r.json" 2> "$OUT/xcd${v}_$r.err" || { echo "bench xcd$v fail"; tail "$OUT/xcd${v}_$r.err"; exit 1; }
    line "$OUT/xcd${v}_$r.json" "xcd$v $r"
  done
done
