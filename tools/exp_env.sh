#!/usr/bin/env bash
# Experiment: bench under env/arg variants.  RUNS="name|ENV=1 ENV2=0|--config c3 --stream-priority 0" ...
# (entries separated by ';')
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
IFS=';' read -ra ITEMS <<< "$RUNS"
for it in "${ITEMS[@]}"; do
  IFS='|' read -r name envs args <<< "$it"
  out=gpurun_out/exp_$name
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --cpu-seconds 0 $args > $out.json 2> $out.err || exit 3
  python3 -c "
import json; d=json.load(open('$out.json'))
print('$name', d['ms_per_step'], {k: round(v, 4) for k, v in d['kernel_ms'].items() if v > 0.006})"
done
