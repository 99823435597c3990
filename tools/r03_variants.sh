#!/usr/bin/env bash
# Bench A/B of library build variants (rvgrt_amd/variants/<v>/): ms/frame per config, two runs each.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in main ${VARIANTS}; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for c in ${CONFIGS:-c4 c3}; do for rep in 1 2; do
    RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 > gpurun_out/var_$v.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/var_$v.json') if l.startswith('{')][-1]; print('$v $c', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done; done
done
