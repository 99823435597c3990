#!/usr/bin/env bash
# Round-3 grouped-frame checks on the GPU box: parity tests, then C3/C4 bench lines per group
# size and the C4 shard probe (each step under its own time limit; stops at the first crash).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"; return $rc; }
for step in "$@"; do
    case $step in
        tests) run gtests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
                   tests/test_gpu_group.py tests/test_gpu_multirank.py "tests/test_gpu_fullsize.py::test_fullsize_pipelined_frames" || exit 3 ;;
        all) run gall 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/ || exit 3 ;;
        bench) for cfg in ${BENCH_CFGS:-c3 c4}; do for g in ${GROUPS_:-0 4 8}; do
                   run b_${cfg}_g$g 300 python bench.py --config $cfg --group $g --cpu-seconds 0 || exit 3
                   grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"avg_launch_ms": [0-9.]*' gpurun_out/b_${cfg}_g$g.log | tr '\n' ' '; echo
               done; done ;;
        shard) for g in ${SHARD_GROUPS:-0 8}; do
                   SHARD_GROUP=$g RV_GI_SHARD_PROBE=1 run shard_g$g 600 python tools/shard_probe.py ${SHARD_CFG:-c4} 1 ${SHARD_T:-64} || exit 3
                   grep "slowest\|whole" gpurun_out/shard_g$g.log
               done ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
