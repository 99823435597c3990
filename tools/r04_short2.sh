#!/usr/bin/env bash
# Round 4: bench.py --settle (settle frames from the start of the camera path, which then starts again):
# short and long runs, several settle lengths; C4 native and drop-in, C3 grouped.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for args in "--steps 20 --warmup 5 --settle 0" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --settle 300" "--steps 20 --warmup 5 --settle 1000" "--steps 200 --warmup 20 --settle 0" "--steps 200 --warmup 20" "--steps 20 --warmup 5 --loop drawcuda --settle 0" "--steps 20 --warmup 5 --loop drawcuda" "--config c3 --steps 24 --warmup 8 --settle 0" "--config c3 --steps 24 --warmup 8"; do
  timeout -k 10 200 python bench.py $args --cpu-seconds 0 > gpurun_out/short.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/short.json') if l.startswith('{')][-1]; print('$args', d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('latency_ms'), d.get('settle_frames'))"
done
