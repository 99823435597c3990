#!/usr/bin/env bash
# Round 4: where the C4 launch's vector-memory (TD) time goes at the round-4 code -- gather coherence per
# site (gdiag build, tools/gather_diag.py) -- and the half-res LDS window for the pipelined render
# (RV_HALF_WINDOW=1) against the product, alternating runs.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
RVGRT_LIB=$PWD/rvgrt_amd/variants/gdiag/librvgrt_hip.so timeout -k 10 400 python tools/gather_diag.py c4 3 > gpurun_out/td_gdiag_c4.txt 2>&1 || { tail -5 gpurun_out/td_gdiag_c4.txt; exit 3; }
head -40 gpurun_out/td_gdiag_c4.txt
for rep in 1 2; do for v in main halfwin; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 200 --cpu-seconds 0 > gpurun_out/td_b.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/td_b.json') if l.startswith('{')][-1]; print('c4 $v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
