#!/bin/bash
# GPU: k_heartbeat<32> instruction counts at C3 (one SQ counter pass,
# kernel-trace only), summed per launch: the VALU-issue roofline's input.
set -uo pipefail
TAG="${1:-pmc_hb}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --kernel-include-regex "k_heartbeat<32>" -d "$OUT/hb_sq" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/hb_sq.log" 2>&1 || { echo "rc=$?"; tail -5 "$OUT/hb_sq.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
f = glob.glob(f"{out}/hb_sq/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
disp = sorted({int(r["Dispatch_Id"]) for r in rows})
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    tot[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for d in disp:
    print("dispatch", d, {k: f"{v:.4g}" for k, v in sorted(tot[d].items())})
last = disp[-3:]   # steady ticks (the timed ones)
for c in sorted(tot[disp[0]]):
    print(f"steady {c} per launch {sum(tot[d][c] for d in last) / len(last):.5g}")
PY
