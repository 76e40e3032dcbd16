#!/bin/bash
# GPU (round 5): the list-driven send on push shards and the split commit shared
# by topic -- shard / c5-shape parity, c5 at 2M on 8 serial shards, serial K=8
# C3 A/B of the split commit (by topic against dealt batches), then a C3 A/B of
# the refresh grid and the commit's slot batch.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05p"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_shard.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { grep -E "^E |FAILED|passed|failed" "$OUT/pytest.log" | head -30; exit 1; }
tail -1 "$OUT/pytest.log"
GSIM_GROUP_SERIAL=1 timeout -k 10 600 python -u bench.py --config c5 --peers 2000000 --shards 8 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c5_2M_s8.json" 2> "$OUT/c5_2M_s8.err" || { echo s8 fail; tail "$OUT/c5_2M_s8.err"; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s=d['kernel_ms_per_tick_shards']; print('c5 2M s8', round(d['ms_per_step'],2), s, 'mean', round(sum(s)/len(s),2), 'max', max(s))
print({x: round(v,1) for x,v in d['kernel_ms_per_tick'].items() if v > 0.05})" "$OUT/c5_2M_s8.json"
LIBS="topic:$L/libgsim.so dealt:$L/libgsim_splitdealt.so" ROUNDS=2 tools/gpu_ab_shards.sh r05p_ab || exit 1
LIBS="base:$L/libgsim.so rg32k:$L/libgsim_rg32k.so rg128k:$L/libgsim_rg128k.so sb16:$L/libgsim_sb16.so sb4:$L/libgsim_sb4.so" \
  ROUNDS=2 STEPS=5 tools/gpu_ab_libs.sh r05p_c3
