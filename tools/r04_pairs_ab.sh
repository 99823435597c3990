#!/usr/bin/env bash
# Round 4: GI lane pairs (RV_GI_PAIRS) on the latency-variant launches: C3 pipelined (--group 0) and C3 drop-in
# (flow launch), two runs each: pairs loop ms/frame launch-ms.
cd "$(dirname "$0")/.." || exit 1
for rep in 1 2; do for pairs in 0 1; do
  RV_GI_PAIRS=$pairs timeout -k 10 200 python bench.py --config c3 --group 0 --steps 300 --cpu-seconds 0 > gpurun_out/pab_n.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/pab_n.json') if l.startswith('{')][-1]; print('pairs $pairs c3 pipelined', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  RV_GI_PAIRS=$pairs timeout -k 10 200 python bench.py --config c3 --loop drawcuda --steps 300 --cpu-seconds 0 > gpurun_out/pab_d.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/pab_d.json') if l.startswith('{')][-1]; print('pairs $pairs c3 drawcuda', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['latency_ms'])"
done; done
