#!/usr/bin/env bash
# A/B of library build variants on the GPU box.  VARIANTS="main g4 g8"
# (main = rvgrt_amd/librvgrt_hip.so, others rvgrt_amd/variants/<v>/).
# Per variant: C2/C3/C4 bench lines (short) and the per-rank tile-share
# render times (tools/host_overhead.py quick).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-main}; do
  lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for cfg in ${CONFIGS:-c2 c3 c4}; do
    out=gpurun_out/var_${v}_${cfg}
    RVGRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-50} --warmup 5 --cpu-seconds 0 \
        > $out.json 2> $out.err || exit 3
    python3 -c "
import json; d=json.load(open('$out.json'))
print('$v $cfg ms', d['ms_per_step'], {k: round(v, 4) for k, v in d['kernel_ms'].items() if v > 0.006}, 'frac', d['roofline']['frac'])"
  done
  if [ "${TILES:-1}" = 1 ]; then
    RVGRT_LIB=$lib timeout -k 10 300 python tools/host_overhead.py ${TILECFG:-c2} quick > gpurun_out/var_${v}_tiles.log 2>&1 || exit 3
    grep "tiles_N\|^frame" gpurun_out/var_${v}_tiles.log | sed "s/^/$v /"
  fi
done
