#!/usr/bin/env bash
# Round 4: what the flow launch costs over the pipelined one -- timing-only builds (wrong frames):
# flownowait (no tag check, no wait), flownofb (wait, but no inline fallback evaluation) -- against the
# product flow launch and the native pipelined loop (look-ahead), same box, two runs each.
cd "$(dirname "$0")/.." || exit 1
for v in main flownowait flownofb; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for rep in 1 2; do
    RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config ${CFG:-c4} --loop drawcuda --steps 200 --cpu-seconds 0 > gpurun_out/fab2_$v.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/fab2_$v.json') if l.startswith('{')][-1]; print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['latency_ms'])"
  done
done
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config ${CFG:-c4} --steps 200 --cpu-seconds 0 > gpurun_out/fab2_pipe.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/fab2_pipe.json') if l.startswith('{')][-1]; print('pipe', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['latency_ms'])"
done
