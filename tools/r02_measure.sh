#!/usr/bin/env bash
# Round-2 measurement batch on one MI355X (gpurun): the driver's default bench line (C4 with the
# CPU baseline), bench lines of C1/C2/C3/C5, a rocprofv3 kernel-trace + stats pass of the default
# bench, and PMC passes (HBM read/write bytes, vector-memory counters) for C4 and C3 that
# tools/pmc_summary.py turns into profiles/traffic_<config>.json.  Each GPU step has its own time
# limit; the batch stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/m_$name.log" 2>&1 || { echo "FAILED $name rc=$?"; tail -5 "gpurun_out/m_$name.log"; exit 3; }; tail -1 "gpurun_out/m_$name.log" | cut -c1-300; }
step bench_c4 300 python bench.py
for c in ${CONFIGS:-c1 c2 c3 c5}; do
  cs=10; [ "$c" = c5 ] && cs=0
  step bench_$c 300 python bench.py --config $c --cpu-seconds $cs
done
rm -rf gpurun_out/prof_c4
step prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python3 bench.py --cpu-seconds 0
for c in ${PMC_CONFIGS:-c4 c3 c2}; do
  for set in "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1)
    rm -rf gpurun_out/pmc_${c}_$tag
    step pmc_${c}_$tag 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc_${c}_$tag -o run -- \
        python3 bench.py --config $c --steps 32 --warmup 8 --cpu-seconds 0
  done
done
echo "== done"
