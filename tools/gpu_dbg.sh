set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug_delivery.py b > gpurun_out/dbg.log 2>&1; tail -30 gpurun_out/dbg.log
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -5 gpurun_out/pt.log
