#!/usr/bin/env bash
# (Record of the round-4 A/B: the cooperative-march code and its variant builds were removed after it;
#  results in profiles/r04/coop_ab.txt.)
# Round 4: the cooperative sphere march of the latency variants (RV_COOP, rv_device.h sphere_coop).
#   1. the GPU suite (every small test frame takes the latency variant) unless TESTS=0;
#   2. per library (main = RV_COOP 1, nocoop): the 8-rank C4 share at one frame per launch (shard_probe),
#      the C3 drop-in line (latency-mode flow frames) and the C4 line (throughput variant: unchanged code);
#   3. wave lifetimes of rank 0 of 8 (diag builds, tools/pipe_waves.py).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/coop_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/coop_tests.log; [ $rc = 0 ] || exit 3
fi
for v in ${VARIANTS:-main nocoop exp1 exp2 max1}; do
  lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  echo "== $v"
  RVGRT_LIB=$lib SHARD_GROUP=0 SHARD_NS=8 RV_GI_SHARD_PROBE=1 timeout -k 10 300 python tools/shard_probe.py c4 1 64 2>&1 | grep "N=8\|whole" || exit 3
  lines="c3_drawcuda"; case $v in main|nocoop) lines="c3_drawcuda c4_native";; esac
  for line in $lines; do set -- ${line/_/ }
    RVGRT_LIB=$lib timeout -k 10 200 python bench.py --config $1 --loop $2 --steps 200 --cpu-seconds 0 > gpurun_out/coop_b.json 2>/dev/null || exit 3
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/coop_b.json') if l.startswith('{')][-1]; print('  $1 $2', d['ms_per_step'], 'lat', d['latency_ms'], d['roofline']['avg_launch_ms'])"
  done
done
for v in diag diagexp1 diagnocoop; do
  echo "== waves $v"
  RVGRT_LIB=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so RV_PIPE_WAVE_STATS=1 RV_GI_SHARD_PROBE=1 timeout -k 10 300 python tools/pipe_waves.py c4 8 64 > gpurun_out/coop_waves_$v.log 2>&1 || exit 3
  grep -h "us/frame\|longest" gpurun_out/coop_waves_$v.log
done
