#!/usr/bin/env bash
# Grouped-launch A/B of library variants: C4 on one GPU at --group 16 and 0 (bench), and the slowest
# 8-rank C4 share at 16 frames per launch (tools/shard_probe.py, 64-px tiles).  VARIANTS="main gw7 ..."
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-main}; do
  lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for g in ${GROUPS_:-16}; do
    RVGRT_LIB=$lib timeout -k 10 240 python bench.py --config ${CFG:-c4} --group $g --cpu-seconds 0 > gpurun_out/gab_${v}_g$g.json 2>/dev/null \
      || { echo "FAILED bench $v"; exit 3; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/gab_${v}_g$g.json') if l.startswith('{')][-1]
print('$v ${CFG:-c4} group $g: ms/frame', d['ms_per_step'], 'kernel', d['roofline']['kernel'], d['roofline']['avg_launch_ms'], 'x', d['roofline']['frames_per_launch'])"
  done
  if [ "${PROBE:-1}" = 1 ]; then
    RVGRT_LIB=$lib SHARD_GROUP=16 SHARD_NS=${SHARD_NS:-8} RV_GI_SHARD_PROBE=1 timeout -k 10 300 python tools/shard_probe.py ${CFG:-c4} 1 64 \
      > gpurun_out/gab_${v}_probe.log 2>&1 || { echo "FAILED probe $v"; exit 3; }
    grep "whole\|slowest" gpurun_out/gab_${v}_probe.log | sed "s/^/$v /"
  fi
done
