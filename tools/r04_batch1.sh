#!/usr/bin/env bash
# Round 4, first GPU batch: flow tests + drop-in bench lines (tools/r04_flow.sh), C4 P1 ablations
# (tools/r04_ablate_p1.sh), C3 GI-texture A/B (table vs noise for the GI bounce hits).  Stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
bash tools/r04_flow.sh || exit 3
echo "== P1 ablations ($(date +%T))"
bash tools/r04_ablate_p1.sh > gpurun_out/r4_ablate_p1.txt 2>&1 || { echo "FAILED ablations"; tail -5 gpurun_out/r4_ablate_p1.txt; exit 3; }
cat gpurun_out/r4_ablate_p1.txt
echo "== C3 GI texture A/B ($(date +%T))"
for v in main gitexnoise main gitexnoise; do lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config c3 --steps 200 --cpu-seconds 0 > gpurun_out/r4_gitex_$v.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r4_gitex_$v.json') if l.startswith('{')][-1]; print('c3 $v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
echo "== batch done ($(date +%T))"
