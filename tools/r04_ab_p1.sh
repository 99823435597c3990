#!/usr/bin/env bash
# Round 4: A/B of render-path variants on C4 P1 (water-heavy) and P0, native loop, two runs each:
# variant pose ms/frame k_ref_pipe-launch-ms.  VARIANTS = main and rvgrt_amd/variants/<name> builds.
cd "$(dirname "$0")/.." || exit 1
for pose in ${POSES:-P1 P0}; do
  for v in ${VARIANTS:-main}; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
    for rep in 1 2; do
      RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config ${CFG:-c4} --pose $pose --steps 100 --cpu-seconds 0 > gpurun_out/abp1_$v.json 2>/dev/null || exit 3
      python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/abp1_$v.json') if l.startswith('{')][-1]; print('$v $pose', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
    done
  done
done
