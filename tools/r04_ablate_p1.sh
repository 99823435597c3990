#!/usr/bin/env bash
# Round 4: ablations of the water-heavy C4 pose P1 (RV_ABLATE builds in rvgrt_amd/variants/abl<bits>/, timing
# experiments only; tools/build_variant.sh): ms/frame and the k_ref_pipe launch time per variant, two runs
# each.  Bits: 1 texture tile, 2 cones, 4 water branch (reflection -> sky), 8 fog, 64 pre-pass part, 32 GI part,
# 2048 the water normal's fbm3D, 4096 the reflection shadow ray, 8192 the reflection ray.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in main ${ABL:-abl1 abl2 abl4 abl8 abl32 abl64 abl2048 abl4096 abl8192}; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for rep in 1 2; do
    RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config ${CFG:-c4} --pose ${POSE:-P1} --steps 100 --cpu-seconds 0 > gpurun_out/ablp1_$v.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/ablp1_$v.json') if l.startswith('{')][-1]; print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
