#!/usr/bin/env bash
# Round 4: rank shares at the final code (tools/shard_probe.py, 64-px tiles, GI shard, no exchange): one frame per
# launch (SHARD_GROUP=0) and 16 per launch, C4 and C5, N = 2, 4, 8.
cd "$(dirname "$0")/.." || exit 1
for c in c4 c5; do for g in 0 16; do
  echo "== $c SHARD_GROUP=$g ($(date +%T))"
  SHARD_GROUP=$g SHARD_NS=2,4,8 RV_GI_SHARD_PROBE=1 timeout -k 10 500 python tools/shard_probe.py $c 1 64 2>&1 | grep -v "frames \.\.\.\|amdgpu.ids" || exit 3
done; done
