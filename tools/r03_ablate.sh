#!/usr/bin/env bash
# Ablation A/B of the pipelined C4 launch (RV_ABLATE builds in rvgrt_amd/variants/abl<bits>/, timing
# experiments only): ms/frame and the k_ref_pipe launch time per variant, two runs each.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in main ${ABL:-abl1 abl2 abl4 abl32 abl64 abl128}; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for rep in 1 2; do
    RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config ${CFG:-c4} --cpu-seconds 0 > gpurun_out/abl_$v.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/abl_$v.json') if l.startswith('{')][-1]; print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
