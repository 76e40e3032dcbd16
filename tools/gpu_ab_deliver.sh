#!/bin/bash
# Delivery ablations + PMC counters of k_send.
set -euo pipefail
TAG="${1:-abd}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u tools/ab_deliver.py > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
tail -1 "$OUT/ab.log"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_send" -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_send" -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_send" -d "$OUT/pmc_atomic" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_atomic.log" 2>&1
echo done
