#!/usr/bin/env bash
# Round 4: the drop-in loop before the flow launch -- rv_update_gi_data + one frame per call, no camera
# look-ahead (bench.py --loop python: renderLoop's UpdateGIData -> drawCUDA order), C3/C4/C5 P0.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for c in ${CFGS:-c4 c3 c5}; do
  echo "== $c ($(date +%T))"
  timeout -k 10 240 python bench.py --config $c --loop python --cpu-seconds 0 ${EXTRA:-} > gpurun_out/r4_base_$c.json 2> gpurun_out/r4_base_$c.log \
    || { echo "FAILED $c rc=$?"; tail -5 gpurun_out/r4_base_$c.log; exit 3; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r4_base_$c.json')); print('$c', d['ms_per_step'], d['kernel_ms'], d['stage_ms'])"
done
echo "== done"
