#!/usr/bin/env bash
# Round-3 measurement batch on one MI355X (gpurun), every GPU step under its own time limit, stopping at
# the first failure:
#   1. PMC passes (FETCH_SIZE, WRITE_SIZE; then TA/TD/TCP/SQ) per config and pose; tools/pmc_summary.py
#      -> profiles/traffic_<cfg>[_P1].json (read by bench.py's roofline.traffic) and gpurun_out/ copies;
#   2. bench lines: C4 (the driver's default, with the CPU baseline), C1-C3 and C5 (CPU baseline
#      stride-16 for 4K), C3/C4/C5 at pose P1 -> gpurun_out/m3_bench_<cfg>[_P1].json;
#   3. rocprofv3 --kernel-trace --stats of the default bench -> gpurun_out/m3_prof_c4/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/m3_$name.log" 2>&1 || { echo "FAILED $name rc=$?"; tail -5 "gpurun_out/m3_$name.log"; exit 3; }; }
# cfg:pose:kernel:frames-per-launch
SPECS=${SPECS:-"c4:P0:k_ref_pipe:1 c3:P0:k_ref_group:8 c5:P0:k_ref_pipe:1 c2:P0:k_render<:16 c1:P0:k_render<:16 c4:P1:k_ref_pipe:1 c3:P1:k_ref_group:8 c5:P1:k_ref_pipe:1"}
if [ "${PMC:-1}" = 1 ]; then
  for spec in $SPECS; do
    IFS=: read c pose kern fpl <<< "$spec"
    tag=${c}_$pose; suf=""; [ "$pose" != P0 ] && suf=_$pose
    for set in "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
      t=$(echo $set | cut -d' ' -f1)
      rm -rf gpurun_out/pmc_m3${tag}_$t
      timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc_m3${tag}_$t -o run -- \
          python3 bench.py --config $c --pose $pose --steps 32 --warmup 8 --cpu-seconds 0 > gpurun_out/m3_pmc_${tag}_$t.log 2>&1 \
          || { echo "FAILED pmc $tag $t"; tail -3 gpurun_out/m3_pmc_${tag}_$t.log; exit 3; }
    done
    python3 tools/pmc_summary.py --prefix m3${tag}_ --config $c$suf --kernel "$kern" --fpl $fpl --grid -1 \
        --out gpurun_out/traffic_$c$suf.json && cp gpurun_out/traffic_$c$suf.json profiles/traffic_$c$suf.json
  done
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench_c4 300 python bench.py
  cp gpurun_out/m3_bench_c4.log gpurun_out/m3_bench_c4.json
  for c in c1 c2 c3 c5; do step bench_$c 300 python bench.py --config $c --cpu-seconds 10; cp gpurun_out/m3_bench_$c.log gpurun_out/m3_bench_$c.json; done
  for c in c3 c4 c5; do step bench_${c}_P1 300 python bench.py --config $c --pose P1 --cpu-seconds 10; cp gpurun_out/m3_bench_${c}_P1.log gpurun_out/m3_bench_${c}_P1.json; done
fi
if [ "${PROF:-1}" = 1 ]; then
  rm -rf gpurun_out/m3_prof_c4
  step prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m3_prof_c4 -o run -- python3 bench.py --cpu-seconds 0
fi
echo "== done"
