#!/bin/bash
# build libgsim variant with extra flags: buildvar.sh NAME "FLAGS"
set -e
cd "$(dirname "$0")/../go-libp2p-pubsub_amd"
N=$1; F=$2
mkdir -p build/v_$N
for s in csrc/*.hip csrc/*.cpp; do
  b=$(basename $s)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -I../include -Icsrc $F -c $s -o build/v_$N/$b.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libgsim_$N.so build/v_$N/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built libgsim_$N.so
