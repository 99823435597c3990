#!/usr/bin/env bash
# (Record of a round-4 A/B; the GI cell order was removed after it, profiles/r04/gi_order_ab.txt.)
# Round 4: the GI cell order of the pipelined launch (k_gi_order, RV_GI_ORDER) -- GPU suite, then alternating
# bench lines with and without it.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gio_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/gio_tests.log; [ $rc = 0 ] || exit 3
fi
for rep in 1 2; do
for line in ${LINES:-c4_P0 c5_P0 c4_P1}; do c=${line%_*}; pose=${line#*_}
for o in 1 0; do
  RV_GI_ORDER=$o timeout -k 10 200 python bench.py --config $c --pose $pose --loop ${LOOP:-native} --steps 200 --cpu-seconds 0 > gpurun_out/gio_b.json 2>/dev/null || exit 3
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/gio_b.json') if l.startswith('{')][-1]; print('$line order=$o', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done; done
