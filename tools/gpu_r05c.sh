#!/bin/bash
# GPU (round 5): the heartbeat's reads attributed per gathered field -- C3
# lines and a PMC pass over k_heartbeat<32> for builds that restore one
# gather each (trk: tracked loaded eagerly, sub: sub[col] gathered, exact:
# every dirty position re-scored) against HEAD (new) and the previous commit
# (prev); then the serial 8-shard C3 line with its rocprof kernel summary.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r05c}"
mkdir -p "$OUT"
cd "$ROOT"
P=go-libp2p-pubsub_amd
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_tick']; print(sys.argv[2], round(d['ms_per_step'],2), {x: round(v,2) for x,v in k.items() if v > 0.05})" "$1" "$2"; }
for arm in ${ARMS:-prev new trk sub exact}; do
  lib="$ROOT/$P/libgsim_$arm.so"; [ "$arm" = new ] && lib="$ROOT/$P/libgsim.so"
  GSIM_LIB="$lib" timeout -k 10 240 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > "$OUT/b_$arm.json" 2> "$OUT/b_$arm.err" || { echo "bench $arm fail"; tail "$OUT/b_$arm.err"; exit 1; }
  line "$OUT/b_$arm.json" "$arm"
  (cd /tmp && TMPDIR=/tmp GSIM_LIB="$lib" timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum \
     --kernel-include-regex "k_heartbeat<32>" -d "$OUT/pmc_$arm" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/pmc_$arm.log" 2>&1) || { echo "pmc $arm fail"; tail -5 "$OUT/pmc_$arm.log"; exit 1; }
  python3 "$ROOT/tools/pmc_parse.py" "$OUT/pmc_$arm.json" "$OUT/pmc_$arm" > /dev/null 2>&1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(sys.argv[2], k, {c: '%.4g' % v for c, v in r.items() if not c.startswith('_')}) for k, r in d.items()]" "$OUT/pmc_$arm.json" "$arm"
done
[ -n "${NO_SHARDS:-}" ] && exit 0
STEPS=3 tools/gpu_shard8.sh "${1:-r05c}_s8"
