#!/usr/bin/env bash
# Experiment: frame-kernel workgroup scheduling modes (RV_SCHED) on C2/C3/C4.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for cfg in ${CONFIGS:-c2 c3 c4}; do
  for s in ${SCHEDS:-0 1 2 3}; do
    RV_SCHED=$s timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 5 --cpu-seconds 0 \
        > gpurun_out/exp_${cfg}_s$s.json 2> gpurun_out/exp_${cfg}_s$s.err || exit 3
    python3 -c "import json,sys; d=json.load(open('gpurun_out/exp_${cfg}_s$s.json')); print('$cfg sched=$s', d['ms_per_step'], 'ms', d['stage_ms'], 'frac', d['roofline']['frac'])"
  done
done
