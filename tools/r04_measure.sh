#!/usr/bin/env bash
# Round-4 measurement batch on one MI355X (gpurun), every GPU step under its own time limit, stopping at
# the first failure:
#   1. PMC passes (FETCH_SIZE, WRITE_SIZE; then TA/TD/TCP/SQ) per spec; tools/pmc_summary.py
#      -> profiles/traffic_<cfg>[_P1][_drawcuda].json (bench.py's roofline.traffic and roofline.limit);
#   2. bench lines: the driver's default (C4 native loop, with the CPU baseline), C1-C3/C5, P1 lines, and
#      renderLoop's own calls (--loop drawcuda: rv_update_gi_data + rv_draw_cuda, one frame per call) for
#      C3/C4/C5 P0 and C4 P1 -> gpurun_out/m4_bench_<name>.json;
#   3. rocprofv3 --kernel-trace --stats of the default bench and of the C4 drawcuda line.
# Subsets: PMC=0 / BENCH=0 / PROF=0, SPECS="...", LINES="...".
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/m4_$name.log" 2>&1 || { echo "FAILED $name rc=$?"; tail -5 "gpurun_out/m4_$name.log"; exit 3; }; }
# cfg:pose:kernel:frames-per-launch:loop
SPECS=${SPECS:-"c4:P0:k_ref_pipe:1:native c4:P0:k_ref_flow:1:drawcuda c3:P0:k_ref_group:8:native c3:P0:k_ref_flow:1:drawcuda c5:P0:k_ref_flow:1:drawcuda c4:P1:k_ref_flow:1:drawcuda c4:P1:k_ref_pipe:1:native"}
if [ "${PMC:-1}" = 1 ]; then
  for spec in $SPECS; do
    IFS=: read c pose kern fpl loop <<< "$spec"
    suf=""; [ "$pose" != P0 ] && suf=_$pose; [ "$loop" = drawcuda ] && suf=${suf}_drawcuda
    tag=${c}${suf}
    for set in "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
      t=$(echo $set | cut -d' ' -f1)
      rm -rf gpurun_out/pmc_m4${tag}_$t
      timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc_m4${tag}_$t -o run -- \
          python3 bench.py --config $c --pose $pose --loop $loop --steps 32 --warmup 8 --cpu-seconds 0 > gpurun_out/m4_pmc_${tag}_$t.log 2>&1 \
          || { echo "FAILED pmc $tag $t"; tail -3 gpurun_out/m4_pmc_${tag}_$t.log; exit 3; }
    done
    python3 tools/pmc_summary.py --prefix m4${tag}_ --config $c$suf --kernel "$kern" --fpl $fpl --grid -1 \
        --out gpurun_out/traffic_$c$suf.json && cp gpurun_out/traffic_$c$suf.json profiles/traffic_$c$suf.json
  done
fi
# name:args
LINES=${LINES:-"c4:--config_c4 dc_c4:--config_c4_--loop_drawcuda dc_c3:--config_c3_--loop_drawcuda dc_c5:--config_c5_--loop_drawcuda dc_c4_P1:--config_c4_--pose_P1_--loop_drawcuda c1:--config_c1 c2:--config_c2 c3:--config_c3 c5:--config_c5 c3_P1:--config_c3_--pose_P1 c4_P1:--config_c4_--pose_P1 c5_P1:--config_c5_--pose_P1"}
if [ "${BENCH:-1}" = 1 ]; then
  for spec in $LINES; do
    name=${spec%%:*}; args=$(echo ${spec#*:} | tr '_' ' ')
    step bench_$name 300 python bench.py $args --cpu-seconds 10
    grep '^{' gpurun_out/m4_bench_$name.log | tail -1 > gpurun_out/m4_bench_$name.json
    python3 -c "import json; d=json.load(open('gpurun_out/m4_bench_$name.json')); print('$name', d['ms_per_step'], 'lat', d['latency_ms'], d['roofline']['kernel'], d['roofline']['frac'], (d['roofline'].get('limit') or {}).get('td_busy'))"
  done
fi
if [ "${PROF:-1}" = 1 ]; then
  rm -rf gpurun_out/m4_prof_c4 gpurun_out/m4_prof_dc_c4
  step prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m4_prof_c4 -o run -- python3 bench.py --cpu-seconds 0
  step prof_dc_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m4_prof_dc_c4 -o run -- python3 bench.py --loop drawcuda --cpu-seconds 0
fi
echo "== done ($(date +%T))"
