#!/usr/bin/env bash
# Round 4: the DDA's empty-column skip (trace COL: no voxel gathers for look-ahead groups above the terrain)
# on the water reflections (main) and also on the GI bounce rays (colgi) against none (nocol), and the
# half-res LDS window (halfwin): GPU suite, then alternating bench lines; gather coherence per site (gdiag).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/col_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/col_tests.log; [ $rc = 0 ] || exit 3
fi
for rep in ${REPS:-1 2}; do
for line in ${LINES:-c4_P1 c4_P0 c3_P1 c5_P1}; do c=${line%_*}; pose=${line#*_}
for v in ${VARIANTS:-main nocol colgi halfwin}; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config $c --pose $pose --loop ${LOOP:-native} --steps 200 --cpu-seconds 0 > gpurun_out/col_b.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/col_b.json') if l.startswith('{')][-1]; print('$line $v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done; done
if [ "${GDIAG:-1}" = 1 ]; then
  RVGRT_LIB=$PWD/rvgrt_amd/variants/gdiag/librvgrt_hip.so timeout -k 10 400 python tools/gather_diag.py c4 3 > gpurun_out/td_gdiag_c4.txt 2>&1 || { tail -5 gpurun_out/td_gdiag_c4.txt; exit 3; }
  head -32 gpurun_out/td_gdiag_c4.txt
fi
