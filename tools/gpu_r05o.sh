#!/bin/bash
# GPU (round 5): c5's shape at 2M peers on one engine and on 8 serial shards
# (per-shard kernel ms per tick, the slowest shard), at HEAD.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r05o"
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py --config c5 --peers 2000000 --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/c5_2M_single.json" 2> "$OUT/c5_2M_single.err" || { echo single fail; tail "$OUT/c5_2M_single.err"; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('single', round(d['ms_per_step'],2), {x: round(v,1) for x,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/c5_2M_single.json"
GSIM_GROUP_SERIAL=1 timeout -k 10 600 python -u bench.py --config c5 --peers 2000000 --shards 8 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c5_2M_s8.json" 2> "$OUT/c5_2M_s8.err" || { echo s8 fail; tail "$OUT/c5_2M_s8.err"; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s=d['kernel_ms_per_tick_shards']; print('s8', round(d['ms_per_step'],2), s, 'mean', round(sum(s)/len(s),2), 'max', max(s))
print({x: round(v,1) for x,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/c5_2M_s8.json"
