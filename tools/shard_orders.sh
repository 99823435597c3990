#!/usr/bin/env bash
# Slowest rank share of a C4 frame at 8 ranks, one frame per launch, per pipelined-launch dispatch order
# (RV_PIPE_ORDER hex digits, first = lowest workgroup ids: 1 pre-pass, 0 GI, 2 render).  On the GPU box.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for o in "$@"; do
    echo "== RV_PIPE_ORDER=$o"
    RV_PIPE_ORDER=$o SHARD_GROUP=0 SHARD_NS=8 RV_GI_SHARD_PROBE=1 timeout -k 10 300 python tools/shard_probe.py c4 1 64 \
        2>&1 | grep -E "whole frame|N=8" || exit 3
done
