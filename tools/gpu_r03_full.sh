#!/bin/bash
# GPU: the -m gpu suite, the default bench line (CPU baselines on), a C3 kernel
# trace with rocprofv3 --stats, and the c5 line; outputs under gpurun_out/TAG.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03full}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && { grep -E "^E |FAILED" "$OUT/pytest_gpu.log" | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
t0=$SECONDS
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
echo "default bench wall: $((SECONDS - t0)) s"
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c3', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'cpu', d['cpu_baseline']['value'])" "$OUT/bench_default.json"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o s -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_c3.log" 2>&1 ) || { tail -20 "$OUT/prof_c3.log"; exit 1; }
python3 "$ROOT/tools/trace_summary.py" "$OUT/prof_c3/s_kernel_trace.csv" 1 6 > "$OUT/prof_c3_summary.txt"; head -12 "$OUT/prof_c3_summary.txt"
timeout -k 10 500 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { tail -20 "$OUT/bench_c5.err"; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', round(d['ms_per_step'],2), {k: round(v,1) for k,v in d['kernel_ms_per_tick'].items() if v > 1})" "$OUT/bench_c5.json"
