#!/bin/bash
# GPU session: parity tests + a short bench (no CPU baseline).
set -euo pipefail
TAG="${1:-quick}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
python3 - "$OUT/bench.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 2), "deliv/s %.3g" % d["msg_edge_deliveries_per_sec"])
print("kernels", {k: round(v, 3) for k, v in d["kernel_ms_per_tick"].items()})
print("per tick", {k: round(v) for k, v in d["deliveries_per_tick"].items()})
PY
