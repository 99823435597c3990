#!/usr/bin/env bash
# Round 4: issue priority for the leading (costliest) workgroups of the pipelined launch (RV_PRIO_BLOCKS): the
# 8-rank C4 share at one frame per launch (tools/shard_probe.py), and the whole C4 frame (bench.py), per value.
cd "$(dirname "$0")/.." || exit 1
for pb in ${PBS:-0 256 1024 4096}; do
  echo "== RV_PRIO_BLOCKS=$pb"
  RV_PRIO_BLOCKS=$pb SHARD_GROUP=0 SHARD_NS=8 RV_GI_SHARD_PROBE=1 timeout -k 10 300 python tools/shard_probe.py c4 1 64 2>&1 | grep "N=8\|whole" || exit 3
  RV_PRIO_BLOCKS=$pb timeout -k 10 200 python bench.py --steps 200 --cpu-seconds 0 > gpurun_out/prio.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/prio.json') if l.startswith('{')][-1]; print('  c4 bench', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
