#!/usr/bin/env bash
# Experiment: bench variants.  RUNS="c3:fused:1 c3:fused:0 ..." (config:path:gi_async)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for r in ${RUNS}; do
  IFS=: read -r cfg path ga var <<< "$r"
  out=gpurun_out/exp_${cfg}_${path}_${ga}_${var:-main}
  lib=""; [ -n "$var" ] && lib=$PWD/rvgrt_amd/variants/$var/librvgrt_hip.so
  RVGRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --path $path --gi-async $ga --steps 30 --warmup 5 \
      --cpu-seconds 0 > $out.json 2> $out.err || exit 3
  python3 -c "
import json; d=json.load(open('$out.json'))
print('$r', d['ms_per_step'], {k: round(v, 4) for k, v in d['kernel_ms'].items() if v > 0.006})"
done
