#!/bin/bash
# GPU (round 5): C3 lines at HEAD, the refresh bisect (round-4-head build in
# ab/r4h, HEAD with the 16384-block refresh grid, HEAD on a network without
# IP lists), arms interleaved; rocprof kernel summary at HEAD.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r05a}"
mkdir -p "$OUT"
cd "$ROOT"
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms_per_tick']; print(sys.argv[2], round(d['ms_per_step'],2), 'refresh', round(k.get('refresh_score',0),3), {x: round(v,2) for x,v in k.items() if v > 0.05})" "$1" "$2"; }
for r in 1 2; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/head_$r.json" 2> "$OUT/head_$r.err" || { echo head fail; tail "$OUT/head_$r.err"; exit 1; }
  line "$OUT/head_$r.json" "head $r"
  (cd ab/r4h && timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/r4h_$r.json" 2> "$OUT/r4h_$r.err") || { echo r4h fail; tail "$OUT/r4h_$r.err"; exit 1; }
  line "$OUT/r4h_$r.json" "r4h $r"
  GSIM_LIB="$ROOT/go-libp2p-pubsub_amd/libgsim_g16k.so" timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/g16k_$r.json" 2> "$OUT/g16k_$r.err" || { echo g16k fail; exit 1; }
  line "$OUT/g16k_$r.json" "g16k $r"
  GSIM_BENCH_NO_IPS=1 timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/noip_$r.json" 2> "$OUT/noip_$r.err" || { echo noip fail; exit 1; }
  line "$OUT/noip_$r.json" "noip $r"
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c3 \
  -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof.json" 2> "$OUT/prof.err" || { echo prof fail; tail "$OUT/prof.err"; exit 1; }
python3 "$ROOT/tools/trace_summary.py" "$OUT/prof/c3_kernel_trace.csv" 1 > "$OUT/prof_summary.txt" 2>&1; head -40 "$OUT/prof_summary.txt"
