#!/usr/bin/env bash
# Round 4: longest / p99 wave of each part of the pipelined launch (diag build, tools/pipe_waves.py) for rank 0's
# share at 8 ranks (64-px tiles, GI shard) without and with the GI lane pairs; then C4 / C5 whole frames with the
# GI texture from the noise (gitexnoise) against the table.
cd "$(dirname "$0")/.." || exit 1
lib=$PWD/rvgrt_amd/variants/diag/librvgrt_hip.so
for pairs in 0 1; do
  echo "== rank 0 of 8, RV_GI_PAIRS=$pairs"
  RVGRT_LIB=$lib RV_GI_PAIRS=$pairs RV_PIPE_WAVE_STATS=1 RV_GI_SHARD_PROBE=1 timeout -k 10 300 python tools/pipe_waves.py c4 8 64 > gpurun_out/r4_waves_$pairs.log 2>&1 || exit 3
  grep -h "us/frame\|longest" gpurun_out/r4_waves_$pairs.log
done
for c in c4 c5; do for rep in 1 2; do for v in main gitexnoise; do lib2=""; [ "$v" != main ] && lib2=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  RVGRT_LIB=$lib2 timeout -k 10 200 python bench.py --config $c --steps 200 --cpu-seconds 0 > gpurun_out/gx4_$v.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/gx4_$v.json') if l.startswith('{')][-1]; print('$c $v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done; done
