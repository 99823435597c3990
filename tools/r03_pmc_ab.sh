#!/usr/bin/env bash
# Round-3 A/B of library build variants with counters (verdict r02 item 4): per variant
# (main = rvgrt_amd/librvgrt_hip.so, others rvgrt_amd/variants/<v>/librvgrt_hip.so) and config,
# a bench line and one PMC pass (SQ_INSTS_VALU, SQ_INSTS_VMEM_RD, TD busy, TCP accesses) over the
# dominant kernel; tools/pmc_ab_summary.py prints the table.  Each GPU step has its own limit; the
# batch stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PMC="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-main}; do
  lib=""; [ "$v" != main ] && lib=$PWD/rvgrt_amd/variants/$v/librvgrt_hip.so
  for cfg in ${CONFIGS:-c3 c4}; do
    tag=${v}_${cfg}
    RVGRT_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --cpu-seconds 0 ${BENCH_ARGS:-} \
        > gpurun_out/pab_$tag.json 2> gpurun_out/pab_$tag.err || { echo "FAILED bench $tag"; tail -3 gpurun_out/pab_$tag.err; exit 3; }
    rm -rf gpurun_out/pmcab_$tag
    RVGRT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/pmcab_$tag -o run \
        -- python3 bench.py --config $cfg --steps 32 --warmup 8 --cpu-seconds 0 ${BENCH_ARGS:-} \
        > gpurun_out/pmcab_$tag.log 2>&1 || { echo "FAILED pmc $tag"; tail -3 gpurun_out/pmcab_$tag.log; exit 3; }
    python3 tools/pmc_ab_summary.py $tag
  done
done
