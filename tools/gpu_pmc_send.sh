#!/bin/bash
# GPU: k_send_tm / k_commit request mix at C3 (one counter group per run,
# kernel-trace only): TCP->TCC read / write / atomic requests and the SQ
# instruction and wait counts, summed per launch.
set -uo pipefail
TAG="${1:-pmc_send}"
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
run send_tcp "k_send_tm|k_commit" TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum && \
run send_sq "k_send_tm|k_commit" SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY || exit 1
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
for grp in ("send_tcp", "send_sq"):
    f = glob.glob(f"{out}/{grp}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(grp, "no counter file"); continue
    tot = collections.defaultdict(float); disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        k = "k_send_tm" if "k_send_tm" in r["Kernel_Name"] else "k_commit"
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for (k, c), v in sorted(tot.items()):
        print(f"{grp} {k} {c} per launch {v / max(1, len(disp[k])):.4g}")
PY
