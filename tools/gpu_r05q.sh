#!/bin/bash
# GPU (round 5): test_gater_network_bit_exact[None-2] at HEAD (twice), at the
# last green revision's build (d9daeaf) and with the old refresh grid.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
OUT="$ROOT/gpurun_out/r05q"
mkdir -p "$OUT"
T='tests/test_gater.py::test_gater_network_bit_exact'
for arm in head1:$L/libgsim.so d9:$L/libgsim_d9.so rg64k:$L/libgsim_rg64k.so head2:$L/libgsim.so; do
  name="${arm%%:*}"; lib="$ROOT/${arm#*:}"
  GSIM_LIB="$lib" timeout -k 10 300 python -u -m pytest "$T" -m gpu -q --timeout 200 --timeout-method thread > "$OUT/$name.log" 2>&1
  echo "$name rc=$? $(tail -1 $OUT/$name.log)"
  grep -E "^E " "$OUT/$name.log" | head -3
done
