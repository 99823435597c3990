#!/usr/bin/env bash
# One measurement script for the GPU box (run through gpurun from the repo root), replacing the per-round
# one-off recipes.  Every GPU step runs under its own time limit; the first failure ends the script.
#
#   tools/measure.sh tests [pytest -k expr]        the -m gpu suite            -> gpurun_out/<TAG>_tests.log
#   tools/measure.sh bench NAME:ARGS ...           bench lines (ARGS with _ for spaces, e.g.
#                                                  c4_P1:--config_c4_--pose_P1)  -> gpurun_out/<TAG>_bench_NAME.json
#   tools/measure.sh pmc CFG:POSE:KERNEL:FPL:LOOP  PMC passes (FETCH_SIZE, WRITE_SIZE, then TA/TD/TCP/SQ) of the
#                                                  same bench loop; tools/pmc_summary.py -> gpurun_out/traffic_*.json (copy to profiles/)
#   tools/measure.sh prof [NAME:ARGS ...]          rocprofv3 --kernel-trace --stats of bench lines
#                                                  (default: the driver's bench and the drop-in loop)
#                                                  -> gpurun_out/<TAG>_prof_NAME/
#   tools/measure.sh ab REPS NAME:ENV:ARGS ...     alternating A/B runs (ENV: VAR=v,VAR2=w or -; ARGS as above),
#                                                  REPS rounds, ms/frame of each        -> gpurun_out/<TAG>_ab.txt
#   tools/measure.sh shard CFG GROUP [NS]          slowest rank share per N (tools/shard_probe.py, 64-px tiles,
#                                                  GI shard, no exchange)               -> gpurun_out/<TAG>_shard.txt
#   tools/measure.sh shard-orders ORDER ...        C4's slowest 8-rank share at one frame per launch per
#                                                  RV_PIPE_ORDER (hex digits, lowest ids first: 1 pre-pass,
#                                                  0 GI, 2 render)                      -> gpurun_out/<TAG>_shard_orders.txt
#   tools/measure.sh pmc-l1 CFG POSE KERNEL        L1/L2/UTCL1 and TD/TCP stall counters of one bench loop's
#                                                  kernel (three --pmc passes)          -> gpurun_out/<TAG>_pmc_l1_CFG.txt
#   tools/measure.sh tile-alone CFG POSE FRAMES    flow-launch timelines (tools/flow_waves.py, the diag build in
#                                                  rvgrt_amd/variants/diag): whole, pre-pass alone, the longest
#                                                  pre-pass tile alone                  -> gpurun_out/<TAG>_fw_*.log
#   tools/measure.sh flow-ablation [CFG POSE N]     the drop-in k_ref_flow itemised: full, no GI window, pre-pass +
#                                                  GI, pre-pass alone, the longest pre-pass tile alone (diag build)
#   tools/measure.sh tile-warm [CFG POSE]          the longest pre-pass tile alone, cold vs its lines left in L2
# TAG (env, default r05) prefixes every output; STEPS/WARMUP (env) size the bench runs (default 200/20).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05}
STEPS=${STEPS:-200}
WARMUP=${WARMUP:-20}
cmd=$1; shift

run() {   # run NAME LIMIT cmd...: output to gpurun_out/TAG_NAME.log, stop the script on failure
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1 || {
        echo "FAILED $name rc=$?"; tail -8 "gpurun_out/${TAG}_$name.log"; exit 3; }
}

summary() {   # one line per bench JSON
    python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
rf = d["roofline"]; lim = rf.get("limit") or {}
di = d.get("dropin") or {}
print(sys.argv[1], d["ms_per_step"], "ms/frame,", "lat", d["latency_ms"], "|", rf["kernel"], "frac", rf["frac"],
      "td", lim.get("td_busy"), "| dropin", di.get("ms_per_step"), di.get("latency_ms"),
      (di.get("roofline") or {}).get("frac"))
EOF
}

case "$cmd" in
tests)
    kargs=(); [ -n "$1" ] && kargs=(-k "$1")
    run tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${kargs[@]}"
    tail -3 "gpurun_out/${TAG}_tests.log" ;;
bench)
    for spec in "$@"; do
        name=${spec%%:*}; args=$(echo "${spec#*:}" | tr '_' ' ')
        run "bench_$name" 300 python bench.py $args --steps "$STEPS" --warmup "$WARMUP"
        grep '^{' "gpurun_out/${TAG}_bench_$name.log" | tail -1 > "gpurun_out/${TAG}_bench_$name.json"
        summary "$name" "gpurun_out/${TAG}_bench_$name.json"
    done ;;
pmc)
    for spec in "$@"; do
        IFS=: read -r c pose kern fpl loop <<< "$spec"
        suf=""; [ "$pose" != P0 ] && suf=_$pose; [ "$loop" = drawcuda ] && suf=${suf}_drawcuda
        t=${c}${suf}
        for set in "FETCH_SIZE" "WRITE_SIZE" \
                   "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
            first=${set%% *}
            rm -rf "gpurun_out/pmc_${TAG}${t}_$first"
            echo "== pmc $t $first ($(date +%T))"
            timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "gpurun_out/pmc_${TAG}${t}_$first" \
                -o run -- python3 bench.py --config "$c" --pose "$pose" --loop "$loop" --steps 32 --warmup 8 \
                --cpu-seconds 0 --dropin-leg 0 > "gpurun_out/${TAG}_pmc_${t}_$first.log" 2>&1 || {
                echo "FAILED pmc $t $first"; tail -3 "gpurun_out/${TAG}_pmc_${t}_$first.log"; exit 3; }
        done
        python3 tools/pmc_summary.py --prefix "${TAG}${t}_" --config "$c$suf" --kernel "$kern" --fpl "$fpl" --grid -1 \
            --out "gpurun_out/traffic_$c$suf.json"   # copy into profiles/ from the merged gpurun_out/
    done ;;
prof)
    [ $# -eq 0 ] && set -- "c4:--steps_20_--warmup_5" "dc_c4:--loop_drawcuda_--steps_20_--warmup_5"
    for spec in "$@"; do
        name=${spec%%:*}; args=$(echo "${spec#*:}" | tr '_' ' ')
        rm -rf "gpurun_out/${TAG}_prof_$name"
        run "prof_$name" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_prof_$name" -o run \
            -- python3 bench.py $args --cpu-seconds 0
        grep '^{' "gpurun_out/${TAG}_prof_$name.log" | tail -1 > "gpurun_out/${TAG}_prof_$name/bench_line.json"
    done ;;
ab)
    reps=$1; shift
    out="gpurun_out/${TAG}_ab.txt"
    for ((i = 0; i < reps; i++)); do
        for spec in "$@"; do
            IFS=: read -r name envs args <<< "$spec"
            args=$(echo "$args" | tr '_' ' ')
            envv=(); [ "$envs" != "-" ] && IFS=, read -r -a envv <<< "$envs"
            run "ab_$name" 300 env "${envv[@]}" python bench.py $args --steps "$STEPS" --warmup "$WARMUP" --cpu-seconds 0 \
                --dropin-leg 0
            ms=$(grep '^{' "gpurun_out/${TAG}_ab_$name.log" | tail -1 | python3 -c \
                 "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['latency_ms'])")
            echo "$i $name ${envs} ${args} :: ms/frame launch_ms latency_ms = $ms" | tee -a "$out"
        done
    done ;;
shard)
    c=$1; g=$2; ns=${3:-2,4,8}
    echo "== shard $c group $g ($(date +%T))" | tee -a "gpurun_out/${TAG}_shard.txt"
    SHARD_GROUP=$g SHARD_NS=$ns RV_GI_SHARD_PROBE=1 timeout -k 10 500 python tools/shard_probe.py "$c" 1 64 \
        > "gpurun_out/${TAG}_shard_${c}_$g.log" 2>&1 || { echo "FAILED shard"; tail -5 "gpurun_out/${TAG}_shard_${c}_$g.log"; exit 3; }
    grep -v "frames \.\.\.\|amdgpu.ids" "gpurun_out/${TAG}_shard_${c}_$g.log" | tee -a "gpurun_out/${TAG}_shard.txt" ;;
shard-orders)
    out="gpurun_out/${TAG}_shard_orders.txt"
    for o in "$@"; do
        echo "== RV_PIPE_ORDER=$o" | tee -a "$out"
        RV_PIPE_ORDER=$o SHARD_GROUP=0 SHARD_NS=8 RV_GI_SHARD_PROBE=1 timeout -k 10 300 python tools/shard_probe.py c4 1 64 \
            > "gpurun_out/${TAG}_shard_order_$o.log" 2>&1 || { echo "FAILED shard order $o"; exit 3; }
        grep -E "whole frame|N=8" "gpurun_out/${TAG}_shard_order_$o.log" | tee -a "$out"
    done ;;
pmc-l1)
    c=$1; pose=${2:-P0}; kern=${3:-k_ref_pipe}; i=0
    for set in "TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_SERIALIZATION_STALL_sum TD_COALESCABLE_WAVEFRONT_sum TD_LOAD_WAVEFRONT_sum GRBM_GUI_ACTIVE" \
               "TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TD_TC_STALL_sum TD_SPI_STALL_sum GRBM_GUI_ACTIVE" \
               "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_LATENCY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
        i=$((i + 1))
        rm -rf "gpurun_out/l1_${TAG}${c}_$i"
        echo "== pmc-l1 $c pass $i ($(date +%T))"
        timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "gpurun_out/l1_${TAG}${c}_$i" -o run \
            -- python3 bench.py --config "$c" --pose "$pose" --steps 32 --warmup 8 --cpu-seconds 0 --dropin-leg 0 \
            > "gpurun_out/${TAG}_l1_${c}_$i.log" 2>&1 || { echo "FAILED pass $i"; tail -3 "gpurun_out/${TAG}_l1_${c}_$i.log"; exit 3; }
    done
    python3 tools/pmc_summary.py --l1 "l1_${TAG}${c}_" --kernel "$kern" > "gpurun_out/${TAG}_pmc_l1_$c.txt" || exit 3
    cat "gpurun_out/${TAG}_pmc_l1_$c.txt" ;;
tile-alone)
    c=${1:-c3}; pose=${2:-P0}; n=${3:-40}
    export RVGRT_LIB=rvgrt_amd/variants/diag/librvgrt_hip.so
    run fw_full 200 python tools/flow_waves.py "$c" "$pose" "$n"
    opts=$(grep LONGEST_TILE_OPTS "gpurun_out/${TAG}_fw_full.log" | awk '{print $2}')
    RV_FLOW_OPTS=4 run fw_alone 200 python tools/flow_waves.py "$c" "$pose" "$n"
    RV_FLOW_OPTS=$opts run fw_tile 200 python tools/flow_waves.py "$c" "$pose" "$n"
    grep -h "launch span\|life\|longest pre-pass" "gpurun_out/${TAG}_fw_full.log" "gpurun_out/${TAG}_fw_alone.log" \
        "gpurun_out/${TAG}_fw_tile.log" ;;
flow-ablation)
    # the drop-in flow launch itemised: full | pre-pass + render (no GI window) | pre-pass +
    # GI window (render exits) | pre-pass alone | the longest pre-pass tile alone on an idle chip
    c=${1:-c3}; pose=${2:-P0}; n=${3:-60}
    export RVGRT_LIB=rvgrt_amd/variants/diag/librvgrt_hip.so
    run fa_full 200 python tools/flow_waves.py "$c" "$pose" "$n"
    run fa_nogi 200 python tools/flow_waves.py "$c" "$pose" "$n" --no-gi
    RV_FLOW_OPTS=16 run fa_ppgi 200 python tools/flow_waves.py "$c" "$pose" "$n"
    RV_FLOW_OPTS=4 run fa_pp 200 python tools/flow_waves.py "$c" "$pose" "$n"
    opts=$(grep LONGEST_TILE_OPTS "gpurun_out/${TAG}_fa_full.log" | awk '{print $2}')
    RV_FLOW_OPTS=$opts run fa_tile 200 python tools/flow_waves.py "$c" "$pose" "$n"
    for m in full nogi ppgi pp tile; do
        echo "== $m"; grep -h "MEAN_LAUNCH\|launch span\|life\|wait\|run \|longest pre-pass\|done at" "gpurun_out/${TAG}_fa_$m.log"
    done ;;
tile-warm)
    # is the longest pre-pass chain memory-latency bound?  The same frame every launch (static camera): the
    # longest tile alone after a 1-frame run (caches hold the world build's lines) against after 20 launches
    # of that tile (its own lines left in L2 / MALL by the previous launch)
    c=${1:-c3}; pose=${2:-P0}
    export RVGRT_LIB=rvgrt_amd/variants/diag/librvgrt_hip.so
    run tw_full 200 python tools/flow_waves.py "$c" "$pose" 20 --static
    opts=$(grep LONGEST_TILE_OPTS "gpurun_out/${TAG}_tw_full.log" | awk '{print $2}')
    RV_FLOW_OPTS=$opts run tw_cold 200 python tools/flow_waves.py "$c" "$pose" 1 --static
    RV_FLOW_OPTS=$opts run tw_warm 200 python tools/flow_waves.py "$c" "$pose" 20 --static
    for m in full cold warm; do
        echo "== $m"; grep -h "MEAN_LAUNCH\|launch span\|longest pre-pass\|done at" "gpurun_out/${TAG}_tw_$m.log"
    done ;;
*)
    echo "usage: tools/measure.sh tests|bench|pmc|prof|ab|shard|shard-orders|pmc-l1|tile-alone|flow-ablation|tile-warm ..."; exit 2 ;;
esac
