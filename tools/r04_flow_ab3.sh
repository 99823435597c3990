#!/usr/bin/env bash
# Round 4: the flow launch's fallback code: main (the render's look-ahead-4 traversal inline), flowfbg1
# (look-ahead 1 inline), flownofb (no fallback evaluation: timing only), and the pipelined loop; two runs each.
cd "$(dirname "$0")/.." || exit 1
for v in main flowfbg1 flownofb; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for rep in 1 2; do
    RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config ${CFG:-c4} --loop drawcuda --steps 200 --cpu-seconds 0 > gpurun_out/fab3_$v.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/fab3_$v.json') if l.startswith('{')][-1]; print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['latency_ms'], d['flow_fallbacks'])"
  done
done
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config ${CFG:-c4} --steps 200 --cpu-seconds 0 > gpurun_out/fab3_pipe.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/fab3_pipe.json') if l.startswith('{')][-1]; print('pipe', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['latency_ms'])"
done
