#!/usr/bin/env bash
# Round 4: one-frame-per-launch rank shares (tools/shard_probe.py, 64-px tiles, GI shard, no exchange) with
# and without the GI lane pairs of the latency-variant launches (RV_GI_PAIRS).
cd "$(dirname "$0")/.." || exit 1
for pairs in ${PAIRS:-0 1}; do
  echo "== RV_GI_PAIRS=$pairs ($(date +%T))"
  RV_GI_PAIRS=$pairs SHARD_GROUP=0 SHARD_NS=${SHARD_NS:-4,8} RV_GI_SHARD_PROBE=1 timeout -k 10 400 python tools/shard_probe.py ${CFG:-c4} 1 64 2>&1 | grep -v "frames \.\.\." || exit 3
done
