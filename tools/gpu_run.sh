#!/usr/bin/env bash
# Runs GPU steps on the gpurun box, each under its own time limit.  Stops at
# the first step that crashes, faults or times out (exit >= 2 for pytest,
# non-zero otherwise); ordinary pytest test failures (exit 1) continue.
#   usage: tools/gpu_run.sh step1 step2 ...   (steps: smoke tests bench prof)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "gpurun_out/$name.log"
    return $rc
}
for step in "$@"; do
    case $step in
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 3 ;;
        tests) run tests 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS_K:+-k "$TESTS_K"}
               rc=$?; [ $rc -le 1 ] || exit 3 ;;
        bench) run bench 600 python bench.py || exit 3 ;;
        bench_c3) run bench_c3 600 python bench.py --config c3 --cpu-seconds 5 || exit 3 ;;
        bench_c2) run bench_c2 600 python bench.py --config c2 --cpu-seconds 5 || exit 3 ;;
        bench_c1) run bench_c1 600 python bench.py --config c1 --cpu-seconds 5 || exit 3 ;;
        bench_c5) run bench_c5 600 python bench.py --config c5 --cpu-seconds 0 --steps 128 || exit 3 ;;
        bench_c4) run bench_c4 600 python bench.py --config c4 --cpu-seconds 0 --steps 128 || exit 3 ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof \
                  -o run -- python3 bench.py --cpu-seconds 0 || exit 3 ;;
        pmc) # PMC_SETS: counter sets separated by ';' (one rocprofv3 pass each)
             sets=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD"}
             IFS=';' read -ra SETS <<< "$sets"
             for ctr in "${SETS[@]}"; do
                 tag=$(echo $ctr | tr ' ' '_' | cut -c1-60)
                 tag=${PMC_TAG:-}$tag
                 run pmc_$tag 600 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc_$tag \
                     -o run -- python3 bench.py --steps 16 --warmup 8 --cpu-seconds 0 ${BENCH_ARGS} || exit 3
             done ;;
        pipe) RUNS=${PIPE_RUNS:-"c3:1:012 c3:0:- c4:1:012 c4:0:- c5:1:012"} run pipe 900 tools/exp_pipe.sh || exit 3 ;;
        waves) # PW_RUNS="c3:0 c5:8:32 ..." (config:nranks[:tile_px])
               for pw in ${PW_RUNS:-c3:0 c4:0 c5:0 c4:4:32 c5:8:32}; do
                   IFS=: read -r pc pn pt <<< "$pw"
                   RVGRT_LIB=$PWD/rvgrt_amd/variants/diag/librvgrt_hip.so RV_PIPE_WAVE_STATS=1 RV_GI_SHARD_PROBE=1 \
                       run waves_${pc}_${pn} 300 python tools/pipe_waves.py $pc $pn ${pt:-32} || exit 3
                   grep -h "us/frame\|longest" gpurun_out/waves_${pc}_${pn}.log
               done ;;
        shard) run shard 300 python tools/shard_probe.py c2 16 ${SHARD_T:-16,32,64} || exit 3 ;;
        shard_c4) run shard_c4 300 python tools/shard_probe.py c4 1 32,64 || exit 3 ;;
        shard_gi) RV_GI_SHARD_PROBE=1 run shard_gi 600 python tools/shard_probe.py ${SHARD_CFG:-c4} 1 ${SHARD_T:-16,32} || exit 3 ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
