#!/usr/bin/env bash
# Experiment: pipelined reference frames.  RUNS="c3:1:012 c3:0:- ..." (config:pipe:RV_PIPE_ORDER)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for r in ${RUNS}; do
  IFS=: read -r cfg pipe order <<< "$r"
  out=gpurun_out/exp_pipe_${cfg}_${pipe}_${order}
  env_order=""; [ "$order" != "-" ] && env_order=$order
  RV_PIPE_ORDER=$env_order timeout -k 10 300 python bench.py --config $cfg --pipe $pipe --steps ${STEPS:-100} \
      --warmup 10 --cpu-seconds 0 > $out.json 2> $out.err || exit 3
  python3 -c "
import json; d=json.load(open('$out.json'))
print('$r', d['ms_per_step'], d['fps'], d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['stage_ms'])"
done
