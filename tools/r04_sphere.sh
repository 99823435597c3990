#!/usr/bin/env bash
# Round 4: the sphere march's loop form (RV_SPHERE_UNROLL1: no 2x unroll; RV_SPHERE_FORM=1: plain early exit)
# on the latency-bound launches (8-rank C4 share at one frame per launch, C3 drop-in) and the throughput lines.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${VARIANTS:-main unroll1 form1 form1u}; do
  lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  echo "== $v"
  RVGRT_LIB=$lib SHARD_GROUP=0 SHARD_NS=8 RV_GI_SHARD_PROBE=1 timeout -k 10 300 python tools/shard_probe.py c4 1 64 2>&1 | grep "N=8" || exit 3
  for line in c3_drawcuda c4_native c3_native; do set -- ${line/_/ }
    RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config $1 --loop $2 --steps 200 --cpu-seconds 0 > gpurun_out/sph_b.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/sph_b.json') if l.startswith('{')][-1]; print('  $1 $2', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done; done
