#!/bin/bash
# Register / LDS use of every kernel in a hipcc object: tools/kernel_regs.sh build/deliver.hip.o
set -euo pipefail
B=/opt/rocm/lib/llvm/bin
d=$(mktemp -d)
cp "$1" "$d/x.o"
(cd "$d" && $B/llvm-objdump --offloading x.o > /dev/null)
$B/llvm-readelf --notes "$d"/x.o.0.hipv4-amdgcn-amd-amdhsa--gfx950 | awk '
  /\.group_segment_fixed_size:/ {lds=$2}
  /\.name:/ {name=$2}
  /\.sgpr_count:/ {sg=$2}
  /\.vgpr_count:/ {vg=$2}
  /\.vgpr_spill_count:/ {sp=$2; printf "%-70s vgpr %4s sgpr %4s spill %s lds %s\n", substr(name,1,70), vg, sg, sp, lds}'
rm -rf "$d"
