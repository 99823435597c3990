#!/usr/bin/env bash
# Round 4: short bench runs (the driver's --steps 20 --warmup 5) against long ones, with and without the
# settle frames (bench.py --settle): the first frames after the set-up run slow.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for args in "--steps 20 --warmup 5 --settle 0" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --settle 0" "--steps 20 --warmup 5" "--steps 200 --warmup 20"; do
  timeout -k 10 200 python bench.py $args --cpu-seconds 0 > gpurun_out/short.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/short.json') if l.startswith('{')][-1]; print('$args', d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('latency_ms'), d.get('settle_frames'))"
done
