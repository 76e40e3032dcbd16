#!/bin/bash
# GPU (round 5): the heartbeat without its per-edge gathers (diagnostic build:
# no estate / score gather at rev[e], no sub gather at col[e]; wrong results)
# against HEAD on C3, to bound what an edge-order copy of them could gain.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
LIBS="base:$L/libgsim.so nogather:$L/libgsim_hbnog.so" ROUNDS=2 STEPS=5 tools/gpu_ab_libs.sh r05s_c3
