#!/bin/bash
# GPU (round 5): k_send_tm's sender table (LDS, one read per edge) against the
# binary search over the forwarders' offsets, by the chunk's forwarder count
# threshold (GSIM_TM_TAB_MIN 256 / 128 / 64 / 0), C3 and serial K=8.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=go-libp2p-pubsub_amd
LIBS="t256:$L/libgsim.so t128:$L/libgsim_tab128.so t64:$L/libgsim_tab64.so t0:$L/libgsim_tab0.so" ROUNDS=2 STEPS=5 tools/gpu_ab_libs.sh r05v_c3 || exit 1
LIBS="t256:$L/libgsim.so t64:$L/libgsim_tab64.so t0:$L/libgsim_tab0.so" ROUNDS=1 tools/gpu_ab_shards.sh r05v_s8
