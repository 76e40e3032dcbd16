#!/bin/bash
# GPU: PMC passes (one counter group per run, kernel-trace only) for
#   * HBM traffic of the dominant kernels (FETCH_SIZE / WRITE_SIZE, separate
#     runs; tools/pmc_traffic.py applies the gfx950 read correction) ->
#     profiles/traffic.json entries c3 (k_refresh_score) and c3:send (k_send_tm);
#   * the heartbeat's instruction mix (VALU vs memory, wait cycles).
set -uo pipefail
TAG="${1:-pmc2}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
run() {
  local name="$1" kre="$2"; shift 2
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -d "$OUT/$name" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run ref_fetch "k_refresh_score" FETCH_SIZE && \
run ref_write "k_refresh_score" WRITE_SIZE && \
run send_fetch "k_send_tm" FETCH_SIZE && \
run send_write "k_send_tm" WRITE_SIZE && \
run hb_sq "k_heartbeat<" SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY && \
run hb_sq2 "k_heartbeat<" SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY || exit 1
python3 "$ROOT/tools/pmc_traffic.py" c3 "k_refresh_score" "$OUT/ref_fetch" "$OUT/ref_write" "$OUT/traffic.json" && \
python3 "$ROOT/tools/pmc_traffic.py" c3:send "k_send_tm" "$OUT/send_fetch" "$OUT/send_write" "$OUT/traffic.json"
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for grp in ("hb_sq", "hb_sq2"):
    agg = collections.defaultdict(list)
    for p in glob.glob(os.path.join(out, grp, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{grp} {k:24s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
PY
