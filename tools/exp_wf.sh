#!/usr/bin/env bash
# Experiment: wavefront vs per-pixel frame path, queue append granularity.
#   RUNS="c2:8:mk c2:8:wf0 ..."  (config:flags:mode, mode mk | wf0 | wf1)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for r in ${RUNS}; do
  IFS=: read -r cfg fl mode <<< "$r"
  fa=""; [ "$fl" = "-" ] || fa="--flags $fl"
  mk=0; enq=1
  case $mode in mk) mk=1 ;; wf0) enq=0 ;; wf1) enq=1 ;; esac
  RV_MEGAKERNEL=$mk RV_WF_ENQ=$enq timeout -k 10 300 python bench.py --config $cfg $fa --steps 30 --warmup 5 \
      --cpu-seconds 0 > gpurun_out/exp_${cfg}_${fl}_${mode}.json 2> gpurun_out/exp_${cfg}_${fl}_${mode}.err || exit 3
  python3 -c "
import json; d=json.load(open('gpurun_out/exp_${cfg}_${fl}_${mode}.json'))
print('$r', d['ms_per_step'], {k: round(v, 4) for k, v in d['kernel_ms'].items() if v > 0.006})"
done
