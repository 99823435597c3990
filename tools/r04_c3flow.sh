#!/usr/bin/env bash
# Round 4: the C3 drop-in (flow) line with the throughput variant forced (RV_PIPE_LATENCY_WAVES=0) against the
# latency variant it takes by default, alternating.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for rep in 1 2; do for lw in default 0; do
  if [ $lw = default ]; then unset RV_PIPE_LATENCY_WAVES; else export RV_PIPE_LATENCY_WAVES=$lw; fi
  for c in c3 c4; do
    timeout -k 10 200 python bench.py --config $c --loop drawcuda --steps 200 --cpu-seconds 0 > gpurun_out/c3f.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/c3f.json') if l.startswith('{')][-1]; print('$c drawcuda latency_waves=$lw', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['latency_ms'])"
  done
done; done
